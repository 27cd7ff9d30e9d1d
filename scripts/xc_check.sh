#!/bin/bash
# halo_exchange = 1 inside the resident call: the local-group and RCCL self-peer tests
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${1:-xc}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_multirank.py tests/test_rccl_self.py -m gpu -v --maxfail=3 --timeout 200 --timeout-method thread > $O/xc_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR" $O/xc_tests.log | tail -30; tail -2 $O/xc_tests.log
exit $rc
