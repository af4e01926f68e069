"""Per-step kernel breakdown of the C5 elastodynamics leg from a rocprofv3
kernel trace (tools/c5_probe.py 128 <steps> mg under `rocprofv3 --kernel-trace
--stats --output-format csv`): the steps are cut at the re-assembly kernel's
kernel that closes each step (k_newmark: the state update after the solve); per
step, the device time of each kernel group and of each node-block SpMV level
(by grid size), the median over the steps after the first (which builds the
structure and the hierarchy).
usage: python tools/c5_trace.py <kernel_trace.csv> [out.json]"""
import collections
import csv
import json
import re
import statistics
import sys

GROUPS = [
    ("reassembly (c0 M + K, RHS)", r"k_assemble_elast|k_apply_bcs|k_lincomb"),
    ("PCG SpMV + p.q (node blocks)", r"k_spmv_blk<3, true"),
    ("multigrid smoothing sweeps (node blocks)", r"k_spmv_blk<3, false, 1>|k_spmv_blk3f<[13]>"),
    ("multigrid residuals (node blocks)", r"k_spmv_blk<3, false, 2>|k_spmv_blk3f<2>"),
    ("multigrid fp32 copy of the fine values", r"k_blk3_to_f32"),
    ("multigrid transfer + scaling", r"k_mg_restrict|k_mg_prolong|k_mg_scale|k_mg_mask|k_mg_fix|k_mg_gemv"),
    ("PCG vectors + reductions", r"k_cg_|k_reduce|k_dot"),
    ("Newmark state update", r"k_newmark"),
]


def group(name):
    for g, rx in GROUPS:
        if re.search(rx, name):
            return g
    return "other"


def main():
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            n = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
            n = re.sub(r"\(.*", "", n)
            if "k_spmv_blk" in n:
                n += f" grid {r['Grid_Size_X']}"
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n))
    rows.sort()
    ends = [i for i, (_, _, n) in enumerate(rows) if re.search(r"k_newmark", n)]
    steps = []
    for a, b in zip([0] + [e + 1 for e in ends[:-1]], [e + 1 for e in ends]):
        acc = collections.defaultdict(float)
        kern = collections.defaultdict(float)
        for s, e, n in rows[a:b]:
            acc[group(n)] += (e - s) / 1e6
            kern[n[:100]] += (e - s) / 1e6
        span = (rows[b - 1][1] - rows[a][0]) / 1e6
        steps.append((span, dict(acc), dict(kern)))
    body = steps[1:] if len(steps) > 1 else steps
    out = {"steps": len(steps), "span_ms_median": statistics.median(s for s, _, _ in body), "groups_ms": {},
           "top_kernels_ms": {}}
    for g in sorted({g for _, a, _ in body for g in a}):
        out["groups_ms"][g] = round(statistics.median(a.get(g, 0.0) for _, a, _ in body), 3)
    names = collections.Counter()
    for _, _, k in body:
        for n, v in k.items():
            names[n] += v
    out["kernel_sum_ms_median"] = round(statistics.median(sum(a.values()) for _, a, _ in body), 3)
    for n, v in names.most_common(16):
        out["top_kernels_ms"][n] = round(v / len(body), 3)
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
