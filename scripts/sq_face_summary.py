#!/usr/bin/env python3
"""Issue / wait summary of the op = 1 kernels from rocprofv3 SQ passes and HBM bytes from FETCH / WRITE passes
over scripts/face_probe.py (scripts/final_evidence.sh mode C). Per kernel instance: dispatches, mean duration, and
per dispatch the counters summed over the device; derived: VALU and LDS instructions per wave, the wave-cycle split
(SQ_WAIT_ANY / SQ_WAVE_CYCLES: waiting on anything; SQ_BUSY_CYCLES per dispatch), HBM bytes (FETCH x2 on gfx950).
usage: sq_face_summary.py SQ1_DIR SQ2_DIR FETCH_DIR WRITE_DIR"""
import collections
import csv
import glob
import re
import sys


def load(d):
    path = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    name = {}
    for r in csv.DictReader(open(path)):
        k = int(r["Dispatch_Id"])
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n = r["Kernel_Name"].replace("pamg::(anonymous namespace)::", "")
        m = re.match(r"(void )?(\w+)(<[^>]*>)?", n)
        name[k] = (m.group(2) + (m.group(3) or "")) if m else n[:60]
        dur[k] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return per, dur, name


agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:5]:
    per, dur, name = load(d)
    for k, c in per.items():
        for cn, v in c.items():
            agg[name[k]][cn].append(v)
        agg[name[k]]["_dur_ns"].append(dur[k])
for kn in sorted(agg, key=lambda n: -sum(agg[n]["_dur_ns"])):
    if not kn.startswith(("k_face", "k_restrict")):
        continue
    a = {cn: sum(v) / len(v) for cn, v in agg[kn].items()}
    waves = a.get("SQ_WAVES", 0) or 1
    out = [f"{kn}: {len(agg[kn]['_dur_ns'])} dispatches over the passes, mean {a['_dur_ns'] / 1e3:.1f} us"]
    if "SQ_WAVES" in a:
        out.append(f"  waves {waves:.0f}; VALU {a['SQ_INSTS_VALU'] / waves:.0f}, VMEM rd {a['SQ_INSTS_VMEM_RD'] / waves:.1f}, "
                   f"VMEM wr {a['SQ_INSTS_VMEM_WR'] / waves:.1f} instructions per wave; wave life "
                   f"{a['SQ_WAVE_CYCLES'] / waves:.0f} cycles, of them waiting on anything {a['SQ_WAIT_ANY'] / a['SQ_WAVE_CYCLES']:.2f}, "
                   f"on an instruction dependency {a['SQ_WAIT_INST_ANY'] / a['SQ_WAVE_CYCLES']:.2f}")
    if "SQ_INSTS_LDS" in a:
        out.append(f"  LDS {a['SQ_INSTS_LDS'] / waves:.0f}, SALU {a['SQ_INSTS_SALU'] / waves:.0f}, SMEM {a['SQ_INSTS_SMEM'] / waves:.0f} "
                   f"per wave; VALU active {a['SQ_ACTIVE_INST_VALU'] / max(1, a['SQ_ACTIVE_INST_ANY']):.2f} of issue-active cycles; "
                   f"GRBM_GUI_ACTIVE {a['GRBM_GUI_ACTIVE']:.0f}")
    if "FETCH_SIZE" in a:
        out.append(f"  HBM fetch {2 * a['FETCH_SIZE'] * 1024 / 1e6:.1f} MB (FETCH_SIZE x2), write {a.get('WRITE_SIZE', 0) * 1024 / 1e6:.1f} MB "
                   f"per dispatch -> {(2 * a['FETCH_SIZE'] + a.get('WRITE_SIZE', 0)) * 1024 / (a['_dur_ns'] * 1e-9) / 1e12:.2f} TB/s")
    print("\n".join(out))
