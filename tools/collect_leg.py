"""Summarise one bench leg's rocprofv3 runs (tools/profile_legs.sh) into profiles/.

usage: python tools/collect_leg.py <leg_dir> <leg> <size> <tag> <kernel_regex>

<leg_dir> holds the leg's passes: trace/ (--kernel-trace --stats), fetch/ (--pmc FETCH_SIZE),
write/ (--pmc WRITE_SIZE) and optionally sq/, lds/ (SQ counters).  Writes
  profiles/<tag>_<leg>_kernel_stats.csv  the rocprofv3 stats summary, verbatim
  profiles/<tag>_<leg>_pmc.txt           per-launch counters of the leg's kernels
  profiles/pmc_<leg>.json                what bench.py reads (roofline.traffic, frac_traffic, profile_kernel_ms)
Per launch = the sum over the kernels matching <kernel_regex> of their mean per dispatch (an
assembly launches each of its instances once).  HBM bytes follow MI355X_MICROARCH.md §HBM:
FETCH_SIZE / WRITE_SIZE are KiB; FETCH_SIZE counts wide streaming reads at half their bytes on
gfx950, so it is doubled: hbm = (2 FETCH_SIZE + WRITE_SIZE) * 1024.
"""
import collections
import csv
import glob
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def trace_means(d, rx):
    """kernel name -> (calls, mean ms) from the stats summary of a --kernel-trace --stats run."""
    files = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    out = {}
    for x in csv.DictReader(open(files[0])) if files else []:
        if rx.search(x["Name"]):
            out[x["Name"]] = (int(x["Calls"]), float(x["AverageNs"]) * 1e-6)
    return out, (files[0] if files else None)


def trace_spans(d, rx, names):
    """Mean per-assembly span (ms) when an assembly launches several matching
    kernels (they may overlap on two streams: the sum of their means would
    count the overlap twice): the k-th dispatch of every kernel belongs to
    assembly k; span = last end - first start.  None for a single kernel."""
    if len(names) < 2:
        return None
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        return None
    per = collections.defaultdict(list)
    for x in csv.DictReader(open(files[0])):
        if x["Kernel_Name"] in names:
            per[x["Kernel_Name"]].append((int(x["Start_Timestamp"]), int(x["End_Timestamp"])))
    n = min(len(v) for v in per.values())
    if n == 0:
        return None
    for v in per.values():
        v.sort()
    spans = [(max(per[k][i][1] for k in per) - min(per[k][i][0] for k in per)) * 1e-6 for i in range(n)]
    return sum(spans) / n


def counters(d, rx):
    """counter -> per-launch value (sum over matching kernels of the mean per dispatch)."""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for x in csv.DictReader(open(f)):
            if rx.search(x["Kernel_Name"]):
                acc[x["Counter_Name"]][x["Kernel_Name"]].append(float(x["Counter_Value"]))
    return {c: sum(sum(v) / len(v) for v in per.values()) for c, per in acc.items()}, \
        {c: {k: len(v) for k, v in per.items()} for c, per in acc.items()}


def main():
    d, leg, size, tag, kr = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4], sys.argv[5]
    rx = re.compile(kr)
    out = os.path.join(ROOT, "profiles")
    means, stats_file = trace_means(os.path.join(d, "trace"), rx)
    if stats_file:
        shutil.copy(stats_file, os.path.join(out, f"{tag}_{leg}_kernel_stats.csv"))
    c, ndisp = {}, {}
    for sub in ("fetch", "write", "sq", "lds"):
        v, n = counters(os.path.join(d, sub), rx)
        c.update(v)
        ndisp.update(n)
    kmean = sum(m for _, m in means.values()) if means else None
    span = trace_spans(os.path.join(d, "trace"), rx, set(means))
    if span is not None:
        kmean = span
    lines = [f"# {tag} {leg} (size {size}): per launch = sum over the kernels matching /{kr}/ of their mean per "
             "dispatch (rocprofv3 --pmc, one pass per counter group)"]
    for k, (calls, m) in sorted(means.items()):
        lines.append(f"kernel {k}: {calls} dispatches, mean {m:.5f} ms (--kernel-trace --stats)")
    if span is not None:
        lines.append(f"per assembly (the k-th dispatch of each kernel; first start to last end): mean {span:.5f} ms")
    for k in sorted(c):
        lines.append(f"{k:32s} {c[k]:.6g}   ({sum(ndisp[k].values())} dispatches)")
    rec = {"leg": leg, "size": size, "world": 1, "tag": tag, "kernel_regex": kr,
           "kernels": {k: {"calls": calls, "mean_ms": m} for k, (calls, m) in means.items()},
           "kernel_mean_ms": kmean}
    fetch, write = c.get("FETCH_SIZE"), c.get("WRITE_SIZE")
    if fetch is not None and write is not None:
        hbm = (2.0 * fetch + write) * 1024.0
        lines.append(f"hbm_bytes_per_launch (2*FETCH_SIZE + WRITE_SIZE) KiB*1024 = {hbm:.6g}")
        if kmean:
            lines.append(f"hbm GB/s at the rocprof mean = {hbm / (kmean * 1e-3) / 1e9:.1f} "
                         f"(frac of 8000: {hbm / (kmean * 1e-3) / 8e12:.4f})")
        rec.update(fetch_kib=fetch, write_kib=write, hbm_bytes_per_launch=int(hbm),
                   method="2*FETCH_SIZE + WRITE_SIZE (KiB), MI355X_MICROARCH.md HBM section")
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_ANY",
              "SQ_WAIT_ANY", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE"):
        if k in c:
            rec[k] = c[k]
    if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"] > 0:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
            if k in c:
                lines.append(f"{k} / SQ_WAVE_CYCLES = {c[k] / c['SQ_WAVE_CYCLES']:.3f}")
    if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_ACTIVE_INST_LDS"):
        lines.append(f"SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS = {c['SQ_LDS_BANK_CONFLICT'] / c['SQ_ACTIVE_INST_LDS']:.3f}")
    with open(os.path.join(out, f"{tag}_{leg}_pmc.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    if rec.get("hbm_bytes_per_launch"):
        with open(os.path.join(out, f"pmc_{leg}.json"), "w") as f:
            json.dump(rec, f, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
