#!/bin/bash
# Session-2 pass: face + multirank + RCCL self tests (a failed test is reported, a crash or hang ends
# the call), the face probe with wave / chain stamps, the 2-rank detached bench (halo_exchange 0 / 1).
# usage: r3s2_check.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${1:-s2}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_face_operator.py tests/test_multirank.py tests/test_rccl_self.py -m gpu -v --maxfail=3 --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR" $O/tests.log | head; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests rc $rc"; exit 1; fi
timeout -k 10 300 python scripts/face_probe.py 5 0 > $O/face_probe.txt 2>&1 || { tail $O/face_probe.txt; exit 1; }
cat $O/face_probe.txt
rm -f $O/wave_stamps.bin $O/chain_stamps.bin
PAMG_WAVE_STAMPS=$O/wave_stamps.bin PAMG_CHAIN_STAMPS=$O/chain_stamps.bin timeout -k 10 300 python scripts/face_probe.py 5 0 > $O/face_probe_stamps.txt 2>&1 || exit 1
python3 scripts/wave_stamps.py $O/wave_stamps.bin > $O/wave_stamps.txt 2>&1; tail -4 $O/wave_stamps.txt
python3 scripts/chain_stamps.py $O/chain_stamps.bin > $O/chain_stamps.txt 2>&1; tail -2 $O/chain_stamps.txt
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29532 bench.py --gpus 2 --steps 20 --warmup 5 --comm detached > $O/mp_detached_2.log 2>&1 || { tail -5 $O/mp_detached_2.log; exit 1; }
grep '^{' $O/mp_detached_2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print('mp2', d['value'], e.get('halo_exchange0_vcycles_per_s'), e.get('halo_exchange1_vcycles_per_s'))"
