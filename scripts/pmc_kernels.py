#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 counter passes (any number of pass directories): dispatches, mean
duration, each counter per dispatch, and the issue-side ratios (SQ_WAVE_CYCLES / SQ_WAIT_ANY /
SQ_BUSY_CYCLES are quad-cycle counts). usage: pmc_kernels.py FILTER DIR [DIR ...]"""
import collections
import csv
import glob
import re
import sys

filt = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(dict)
for d in sys.argv[2:]:
    for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"]
            if filt not in name:
                continue
            m = re.search(r"(k_\w+<[^>]*>|k_\w+)", name)
            key = m.group(1) if m else name[:90]
            k = (d, int(r["Dispatch_Id"]))
            agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[key][k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
for key in sorted(agg):
    c = {n: sum(v) / len(v) for n, v in agg[key].items()}
    ds = list(dur[key].values())
    print(f"== {key}: {len(ds)} dispatches (all passes), mean {sum(ds) / len(ds):.4f} ms")
    print("   " + "  ".join(f"{n}={v:.4g}" for n, v in sorted(c.items())))
    if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
        wc = c["SQ_WAVE_CYCLES"]
        parts = [f"{n[3:].lower()} {c[n] / wc:.2f}" for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU",
                                                           "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS") if n in c]
        if "SQ_WAVES" in c and c["SQ_WAVES"]:
            parts.append(f"wave lifetime {4 * wc / c['SQ_WAVES']:.0f} cycles")
            if "SQ_INSTS_VALU" in c:
                parts.append(f"VALU instrs/wave {c['SQ_INSTS_VALU'] / c['SQ_WAVES']:.0f}")
            if "SQ_INSTS_LDS" in c:
                parts.append(f"LDS instrs/wave {c['SQ_INSTS_LDS'] / c['SQ_WAVES']:.0f}")
        print("   " + "  ".join(parts))
