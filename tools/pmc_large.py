"""PMC summary of one kernel's LARGE dispatches only (grid >= min_grid work
items: the C2-size launches of a probe that also runs small cases): per
counter the mean over those dispatches, plus HBM bytes = (2 FETCH_SIZE +
WRITE_SIZE) KiB (MI355X_MICROARCH.md, gfx950).
usage: python tools/pmc_large.py <pmc_dir> <kernel_substring> <min_grid> [title]"""
import collections
import csv
import glob
import sys

d, ksub, min_grid = sys.argv[1], sys.argv[2], int(sys.argv[3])
title = sys.argv[4] if len(sys.argv) > 4 else ""
vals = collections.defaultdict(list)
for f in sorted(glob.glob(d + "/*/run_counter_collection.csv")):
    disp = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if ksub not in r["Kernel_Name"]:
            continue
        key = (r["Kernel_Name"], r["Dispatch_Id"])
        disp[key][r["Counter_Name"]] = disp[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        disp[key]["_grid"] = float(r.get("Grid_Size") or 0)
    for (k, _), c in disp.items():
        if c["_grid"] >= min_grid:
            name = k.replace("(anonymous namespace)::", "").split("(")[0]
            for n, v in c.items():
                if n != "_grid":
                    vals[(name, n)].append(v)
if title:
    print(f"# {title}")
names = sorted({k for k, _ in vals})
for name in names:
    print(name)
    cs = {n: sum(v) / len(v) for (k, n), v in vals.items() if k == name}
    for n in sorted(cs):
        print(f"   {n:28s} n={len(vals[(name, n)]):3d} mean={cs[n]:.4g}")
    if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
        print(f"   hbm_bytes_per_launch (2*FETCH_SIZE + WRITE_SIZE)*1024 = {(2 * cs['FETCH_SIZE'] + cs['WRITE_SIZE']) * 1024:.4g}")
    if "SQ_WAIT_ANY" in cs and "SQ_WAVE_CYCLES" in cs:
        print(f"   SQ_WAIT_ANY / SQ_WAVE_CYCLES = {cs['SQ_WAIT_ANY'] / cs['SQ_WAVE_CYCLES']:.3f}")
