"""Turn a rocprofv3 output tree (tools/profile_r1.sh) into committed summaries.

usage: python tools/collect_profiles.py <prof_dir> <tag> [n]
writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats summary, verbatim),
       profiles/<tag>_pmc.txt           (mean per-dispatch counters of the assembly kernel),
       profiles/pmc_assembly_C2.json    (HBM bytes per launch for bench.py's roofline.traffic)
HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB; FETCH_SIZE counts
128-B requests at 64 B for wide streaming reads on gfx950, so it is doubled; WRITE_SIZE is exact for
16-B-per-lane stores.  Passes are separate rocprofv3 runs.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(d, kernel=("k_assemble_strip", "k_assemble_stencil", "k_assemble_cubes")):
    """Per assembly: the mean per dispatch of each matching kernel, summed over
    the kernels (the assembly launches a uniform-strip and a general instance)."""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True):
        for x in csv.DictReader(open(f)):
            if any(k in x["Kernel_Name"] for k in kernel):
                acc[x["Counter_Name"]][x["Kernel_Name"]].append(float(x["Counter_Value"]))
    return {c: sum(sum(v) / len(v) for v in per.values()) for c, per in acc.items()}


def main():
    prof, tag = sys.argv[1], sys.argv[2]
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 215
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = glob.glob(os.path.join(prof, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(out, f"{tag}_kernel_stats.csv"))
    c = {}
    for sub in ("pmc_sq", "pmc_fetch", "pmc_write", "pmc_lds"):
        c.update(counters(os.path.join(prof, sub)))
    lines = [f"# {tag}: per assembly = sum over the assembly kernels (k_assemble_cubes, or the k_assemble_stencil / k_assemble_strip instances) of their mean per dispatch "
             "(rocprofv3 --pmc, separate passes)"]
    for k in sorted(c):
        lines.append(f"{k:32s} {c[k]:.6g}")
    fetch = c.get("FETCH_SIZE")
    write = c.get("WRITE_SIZE")
    if fetch is not None and write is not None:
        hbm = (2.0 * fetch + write) * 1024.0
        lines.append(f"hbm_bytes_per_launch (2*FETCH_SIZE + WRITE_SIZE) KiB*1024 = {hbm:.6g}")
        pj = "pmc_assembly_C2.json" if n == 215 else f"pmc_assembly_n{n}.json"
        with open(os.path.join(out, pj), "w") as f:
            json.dump({"n": n, "world": 1, "tag": tag, "fetch_kib": fetch, "write_kib": write,
                       "hbm_bytes_per_launch": int(hbm),
                       "method": "2*FETCH_SIZE + WRITE_SIZE (KiB), MI355X_MICROARCH.md HBM section"}, f, indent=1)
    with open(os.path.join(out, f"{tag}_pmc.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
