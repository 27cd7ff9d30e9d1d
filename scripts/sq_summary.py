#!/usr/bin/env python3
"""Issue-side summary of a rocprofv3 SQ / GRBM counter pass over scripts/res_pmc.py (the
resident call): per k_vc_resb dispatch the raw counters, the effective clock, VALU
wave-instructions per V-cycle and per tile, VALU busy and the wave-cycle split.
usage: sq_summary.py PASS_DIR [cycles_per_call] [n_tiles] [n_cu]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
cycles = int(sys.argv[2]) if len(sys.argv) > 2 else 200
tiles = int(sys.argv[3]) if len(sys.argv) > 3 else 8192
ncu = int(sys.argv[4]) if len(sys.argv) > 4 else 256
path = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
disp = collections.defaultdict(dict)
meta = {}
for r in csv.DictReader(open(path)):
    if "k_vc_res" not in r["Kernel_Name"]:
        continue
    k = int(r["Dispatch_Id"])
    disp[k][r["Counter_Name"]] = disp[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    meta[k] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["VGPR_Count"], r["Scratch_Size"])
for k in sorted(disp):
    c, (t0, t1, vg, sc) = disp[k], meta[k]
    dur = (t1 - t0) * 1e-9
    print(f"dispatch {k}: {dur * 1e3:.3f} ms ({cycles} cycles), VGPR {vg}, scratch {sc}")
    for n in sorted(c):
        print(f"   {n:22s} {c[n]:.4g}")
    if "GRBM_GUI_ACTIVE" in c:
        clk = c["GRBM_GUI_ACTIVE"] / 8 / dur
        print(f"   effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration): {clk / 1e9:.3f} GHz")
        if "SQ_ACTIVE_INST_VALU" in c:
            busy = c["SQ_ACTIVE_INST_VALU"] * 4 / (ncu * 4 * c["GRBM_GUI_ACTIVE"] / 8)
            print(f"   VALU busy (SQ_ACTIVE_INST_VALU quad-cycles x 4 / ({ncu * 4} SIMDs x cycles)): {busy:.3f}")
    if "SQ_INSTS_VALU" in c:
        v = c["SQ_INSTS_VALU"] / cycles
        print(f"   VALU wave-instructions per V-cycle: {v / 1e6:.2f} M ({v / tiles:.0f} per tile)")
    if "SQ_WAVE_CYCLES" in c and "SQ_WAIT_ANY" in c:
        w = c["SQ_WAVE_CYCLES"]
        act = c.get("SQ_ACTIVE_INST_ANY", 0.0)
        print(f"   wave cycles: active {act / w:.2f}, parked (WAIT_ANY) {c['SQ_WAIT_ANY'] / w:.2f}, "
              f"issue-stalled (WAIT_INST_ANY) {c.get('SQ_WAIT_INST_ANY', 0.0) / w:.2f}")
