#!/bin/bash
# round 6: the whole GPU suite (agglomeration, pruned switches, new goldens), one process
set -o pipefail
timeout -k 10 1050 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r6_full.log 2>&1
