#!/usr/bin/env python3
"""Per-kernel table of rocprofv3 PMC passes (scripts/pmc_sq.sh output). usage: pmc_table.py TAG [kernel-substr]"""
import collections
import csv
import glob
import sys

tag = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "k_vc"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in glob.glob(f"gpurun_out/{tag}_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("pamg::(anonymous namespace)::", "").split("(")[0]
        if sub not in name:
            continue
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print("==", k)
    for c, v in sorted(d.items()):
        print(f"  {c:24s} {sum(v) / len(v):16.1f}  (n={len(v)})")
