#!/bin/bash
# Generic resident kernel (k_vc_res: n_split < 5 or L = 2): in-tree vs scripts/ablibs A/B on
# S = 3 / 4 (L = 3) and S = 5 (L = 2), then all GPU tests. usage: res_generic_check.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-gen}
cd $R && mkdir -p gpurun_out
for rep in 1 2; do
  r=$(timeout -k 10 120 python scripts/ab_probe.py 3,3,3,1 4,3,3,1 5,2,3,1 2>/dev/null) || exit 1
  echo "in-tree: $r" >> gpurun_out/gen_$TAG.txt
  for f in scripts/ablibs/*.so; do
    r=$(PAMG_LIB=$PWD/$f timeout -k 10 120 python scripts/ab_probe.py 3,3,3,1 4,3,3,1 5,2,3,1 2>/dev/null) || exit 1
    echo "$(basename $f): $r" >> gpurun_out/gen_$TAG.txt
  done
done
cat gpurun_out/gen_$TAG.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gen_tests_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/gen_tests_$TAG.log
exit $rc
