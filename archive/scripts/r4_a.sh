#!/bin/bash
# Round-4 first pass: every GPU test (incl. the face operator at bench.py's op=1 configuration and the
# forced 8-byte snapshot), smoke, the bench, then the face probe under rocprofv3 -- first without the
# cooperative chain (PAMG_FACE_CHAIN=0), then with it (the form that crashed at exit in round 3), each
# writing its /proc/self/maps so the crash PCs resolve to a library and offset.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${1:-r4a}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail=5 -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR" $O/gpu_tests.log | head -20; tail -2 $O/gpu_tests.log
if [ $rc -ne 0 ]; then echo "tests rc $rc"; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d.get('extra',{}); print('bench', d['value'], d['roofline']['frac'], (e.get('op1') or {}).get('vcycles_per_s'))"
cd /tmp && export TMPDIR=/tmp
PAMG_FACE_CHAIN=0 PAMG_PROBE_MAPS=$O/maps_nochain.txt timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_face_nochain -o run -- python3 $R/scripts/face_probe.py 5 0 > $O/prof_face_nochain.log 2>&1
echo "face rocprof (no chain) exit $?"
PAMG_PROBE_MAPS=$O/maps_chain.txt timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_face -o run -- python3 $R/scripts/face_probe.py 5 0 > $O/prof_face.log 2>&1
echo "face rocprof (chain) exit $?"
tail -30 $O/prof_face.log
