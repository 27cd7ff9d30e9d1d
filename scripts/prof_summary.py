#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats output directory (sqlite .db or
csv) into a small text table for profiles/. Usage: prof_summary.py DIR [OUT]"""
import csv
import glob
import os
import sqlite3
import sys


def rows_from_db(path):
    con = sqlite3.connect(path)
    cur = con.cursor()
    return [(r[0], int(r[1]), float(r[2]), float(r[3]), float(r[4]))   # top_kernels view: microseconds
            for r in cur.execute("select name, total_calls, total_duration, average, percentage from top_kernels")]


def rows_from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) * 1e-3,
                        float(r["AverageNs"]) * 1e-3, float(r["Percentage"])))
    return out


def main():
    d = sys.argv[1]
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    csvs = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    rows = rows_from_csv(csvs[0]) if csvs else rows_from_db(dbs[0])
    lines = [f"{'kernel':70s} {'calls':>6s} {'total_us':>11s} {'avg_us':>9s} {'pct':>6s}"]
    for name, n, tot, avg, pct in rows:
        short = name.replace("pamg::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        lines.append(f"{short[:70]:70s} {n:6d} {tot:11.1f} {avg:9.2f} {pct:6.2f}")
    text = "\n".join(lines) + "\n"
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
