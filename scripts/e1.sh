set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 120 python scripts/vc_probe.py 5,3,4,15 5,3,4,1 > gpurun_out/e1_base.txt 2>&1 && \
PAMG_DIAG_NOCASCADE=1 timeout -k 10 120 python scripts/vc_probe.py 5,3,4,15 5,3,4,1 > gpurun_out/e1_nocasc.txt 2>&1 && \
PAMG_DIAG_NOCASCADE=1 timeout -k 10 120 python scripts/stamp_probe.py 5 3 > gpurun_out/e1_stamps.txt 2>&1
