#!/usr/bin/env python3
"""Per-(kernel, grid size) durations from a rocprofv3 kernel_trace.csv."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
path = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"].replace("pamg::(anonymous namespace)::", "").split("(")[0]
    acc[(name, int(r["Grid_Size_X"]), int(r["LDS_Block_Size"]), int(r["VGPR_Count"]))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
print(f"{'kernel':34s} {'grid':>9s} {'lds':>6s} {'vgpr':>4s} {'n':>4s} {'avg_us':>8s} {'min_us':>8s}")
for (n, g, l, v), t in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    print(f"{n[:34]:34s} {g:9d} {l:6d} {v:4d} {len(t):4d} {sum(t)/len(t):8.2f} {min(t):8.2f}")
