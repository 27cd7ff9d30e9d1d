set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for d in 0 1 3 0; do PAMG_DIAG=$d timeout -k 10 60 python scripts/vc_probe.py 5,3,4,15 > gpurun_out/diag_$d.txt 2>&1 || exit 1; echo "diag $d: $(grep -v amdgpu gpurun_out/diag_$d.txt)"; done
