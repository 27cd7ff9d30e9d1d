#!/bin/bash
# round 6, last sources: final_evidence.sh modes A (smoke, bench lines, strong and partition probes, 2 detached
# ranks) and B (rocprofv3 kernel stats, PMC passes) in one call
set -o pipefail
bash scripts/final_evidence.sh "$1" A && bash scripts/final_evidence.sh "$1" B
