set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
echo "host: $(hostname) nproc=$(nproc)" > gpurun_out/env.txt
rocm-smi --showproductname >> gpurun_out/env.txt 2>&1 || true
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench1.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof1 -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $R/gpurun_out/prof1.log 2>&1
echo "exit $?"
