#!/usr/bin/env python3
"""HBM bytes per dispatch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KiB) reports
half the bytes of wide coalesced streaming reads -> x2; WRITE_SIZE (KiB) is exact
for 16-B-per-lane streaming stores. Usage:
  pmc_summary.py FETCH_DIR WRITE_DIR OUT_JSON N_SPLIT [alg_bytes_per_launch] [kernel_prefix] [levels] [commit]
kernel_prefix selects the roofline kernel (default "k_vc_fine", the fused V-cycle's
level-1 launch; "void k_smooth<false, true>" for the per-step level-1 smoother)."""
import collections
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


SKIP_DIGEST = ("pamg_face.hip", "pamg_mesh.cpp", "pamg_vtu.cpp")


def source_digest():
    """the kernel sources the counters were measured on (bench.py source_digest: the same hash)"""
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "p-a_multigrids_amd", "csrc")
    # every source the op = 0 kernels and their launch path are built from: all of csrc but the face
    # operator's kernels (pamg_face.hip), the mesh reader and the VTU writer, which none of them uses
    files = sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".h", ".cpp")) and f not in SKIP_DIGEST)
    for f in files + ["../../include/pamg.h"]:
        h.update(f.encode())
        h.update(open(os.path.join(csrc, f), "rb").read())
    return h.hexdigest()[:16]


def per_kernel(d, counter):
    path = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].replace("pamg::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")
        name = name.split("(")[0]
        acc[(name, int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return acc


def main():
    fdir, wdir, out, nsplit = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    alg = float(sys.argv[5]) if len(sys.argv) > 5 and sys.argv[5] else None
    prefix = sys.argv[6] if len(sys.argv) > 6 else "k_vc_fine"
    f = per_kernel(fdir, "FETCH_SIZE")
    w = per_kernel(wdir, "WRITE_SIZE")
    rows = []
    for key in sorted(set(f) | set(w), key=lambda k: -(sum(f.get(k, [0])) + sum(w.get(k, [0])))):
        fk = sum(f.get(key, [0])) / max(1, len(f.get(key, [])))
        wk = sum(w.get(key, [0])) / max(1, len(w.get(key, [])))
        rows.append(dict(kernel=key[0], grid=key[1], fetch_bytes=2 * fk * 1024, write_bytes=wk * 1024,
                         hbm_bytes=2 * fk * 1024 + wk * 1024, n=len(f.get(key, []))))
    smooth = [r for r in rows if r["kernel"].replace("void ", "").startswith(prefix.replace("void ", ""))]
    smooth.sort(key=lambda r: -r["grid"])
    res = {"n_split": nsplit, "levels": int(sys.argv[7]) if len(sys.argv) > 7 else 3, "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), WRITE_SIZE x1, KiB->B",
           "commit": sys.argv[8] if len(sys.argv) > 8 else None, "source_digest": source_digest(),
           "kernels": rows}
    if smooth:
        res["hbm_bytes_per_launch"] = smooth[0]["hbm_bytes"]
        res["kernel"] = smooth[0]
        if alg:
            res["alg_bytes_per_launch"] = alg
            res["traffic_over_alg"] = smooth[0]["hbm_bytes"] / alg
    json.dump(res, open(out, "w"), indent=1)
    for r in rows[:12]:
        print(f"{r['kernel'][:36]:36s} {r['grid']:9d} fetch {r['fetch_bytes']/1e6:9.1f} MB  write {r['write_bytes']/1e6:9.1f} MB")
    if smooth:
        print(prefix, "hbm bytes/launch", smooth[0]["hbm_bytes"], res.get("traffic_over_alg"))


if __name__ == "__main__":
    main()
