#!/usr/bin/env python3
"""The timed call's dispatch in a rocprofv3 kernel trace of bench.py: bench.py's timed pamg_vcycle call is the
last dispatch of the resident kernel (the side measurements and the warm-up come before it). Prints every
dispatch of the kernels whose name starts with PREFIX (default the bench's resident instance) and the last one's
duration, to set beside the bench line's roofline.ms_per_launch (HIP events on the same launch).
Usage: trace_timed.py TRACE_DIR [PREFIX] [BENCH_LOG]"""
import csv
import glob
import json
import sys

d = sys.argv[1]
prefix = sys.argv[2] if len(sys.argv) > 2 else "void pamg::(anonymous namespace)::k_vc_resb<5, 3"
path = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(path)) if r["Kernel_Name"].startswith(prefix)]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    print(f"dispatch {r['Dispatch_Id']:>7s} grid {r['Grid_Size_X']:>8s} {dur:9.4f} ms  {r['Kernel_Name'][:90]}")
if rows:
    last = rows[-1]
    dur = (int(last["End_Timestamp"]) - int(last["Start_Timestamp"])) * 1e-6
    print(f"timed call (last dispatch): {dur:.4f} ms")
    if len(sys.argv) > 3:
        line = [l for l in open(sys.argv[3]) if l.startswith("{")][-1]
        b = json.loads(line)
        ev = b["roofline"]["ms_per_launch"]
        print(f"bench line: roofline.ms_per_launch {ev:.4f} ms (events, the same launch), ratio rocprof / events "
              f"{dur / ev:.3f}; value {b['value']} V-cycles/s, frac {b['roofline']['frac']}")
