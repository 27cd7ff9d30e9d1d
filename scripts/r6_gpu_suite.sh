#!/bin/bash
# the whole GPU suite, one process (the round-end driver's form)
set -o pipefail
timeout -k 10 1050 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r6_suite_final.log 2>&1
