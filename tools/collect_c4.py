"""Profiles of the C4 leg (tools/profile_r1.sh with B='bench.py --legs c4 ...'): the run also
assembles C2 first, so the C4 dispatches are taken as the last `n_c4` of each assembly kernel
(the leg's warmup + reps), per PMC pass; the kernel durations from the trace likewise.
usage: python tools/collect_c4.py <prof_dir> <tag> [n_c4=7]"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("k_assemble_stencil", "k_assemble_strip", "k_assemble_cubes")


def main():
    prof, tag = sys.argv[1], sys.argv[2]
    n_c4 = int(sys.argv[3]) if len(sys.argv) > 3 else 7
    tot = collections.defaultdict(float)
    for sub in ("pmc_sq", "pmc_fetch", "pmc_write", "pmc_lds"):
        for f in glob.glob(os.path.join(prof, sub, "**", "run_counter_collection.csv"), recursive=True):
            seq = collections.defaultdict(list)
            for r in csv.DictReader(open(f)):
                k = next((x for x in KERNELS if x in r["Kernel_Name"]), None)
                if k:
                    seq[(k, r["Counter_Name"])].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
            for (k, c), v in seq.items():
                v.sort()
                last = [x for _, x in v[-n_c4:]]
                tot[c] += sum(last) / len(last)
    lines = [f"# {tag}: C4 (n=463, 99.9 M DoF, one GPU) -- per assembly = sum over k_assemble_stencil / "
             f"k_assemble_strip of the mean of their last {n_c4} dispatches (the C4 leg; rocprofv3 --pmc, separate passes)"]
    for c in sorted(tot):
        lines.append(f"{c:32s} {tot[c]:.6g}")
    hbm = (2.0 * tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) * 1024.0
    lines.append(f"hbm_bytes_per_launch (2*FETCH_SIZE + WRITE_SIZE) KiB*1024 = {hbm:.6g}")
    tr = glob.glob(os.path.join(prof, "trace", "**", "*kernel_trace.csv"), recursive=True)[0]
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(tr)):
        k = next((x for x in KERNELS if x in r["Kernel_Name"]), None)
        if k:
            dur[k].append((int(r["Dispatch_Id"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    for k, v in dur.items():
        v.sort()
        last = [x for _, x in v[-n_c4:]]
        lines.append(f"kernel_ms {k:26s} mean {sum(last) / len(last):.4f} of the last {n_c4}: "
                     + " ".join(f"{x:.3f}" for x in last))
    out = os.path.join(ROOT, "profiles", f"{tag}_pmc.txt")
    open(out, "w").write("\n".join(lines) + "\n")
    with open(os.path.join(ROOT, "profiles", "pmc_assembly_n463.json"), "w") as f:
        json.dump({"n": 463, "world": 1, "tag": tag, "fetch_kib": tot["FETCH_SIZE"], "write_kib": tot["WRITE_SIZE"],
                   "hbm_bytes_per_launch": int(hbm),
                   "method": "2*FETCH_SIZE + WRITE_SIZE (KiB), MI355X_MICROARCH.md HBM section; last dispatches = C4"},
                  f, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
