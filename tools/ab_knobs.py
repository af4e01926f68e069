"""A/B of assembly kernel variants (afem_set_variant knobs) on one generator
box, in one process, at settled clocks: each round runs every variant as the
bench does -- back to back for --settle ms, then --reps launches bracketed by
HIP events with no synchronisation between them -- and the rounds rotate the
variants.  Prints each variant's median over all rounds and its values'
largest difference from the first variant's (0 = bitwise equal).

usage: python tools/ab_knobs.py [--n 215] [--rounds 4] [--reps 20] [--settle 100]
                                 'A: KNOB=v,KNOB2=v' 'B: KNOB=w' ..."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=215)
ap.add_argument("--nz", type=int, default=None)
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--settle", type=float, default=100.0)
ap.add_argument("--mesh", choices=("box", "arrays", "natural"), default="box",
                help="box: the generator's; arrays: the same box handed over in a random numbering (c2_arrays); "
                     "natural: handed over in its own lexicographic numbering (c2_arrays_natural)")
ap.add_argument("variants", nargs="+")
a = ap.parse_args()

variants = []
for v in a.variants:
    name, _, kv = v.partition(":")
    knobs = dict(x.strip().split("=") for x in kv.split(",") if "=" in x)
    variants.append((name.strip(), knobs))
all_knobs = sorted({k for _, kn in variants for k in kn})

ctx = af.Context(0)
mesh = af.Mesh.structured(ctx, 3, a.n, nz=a.nz, jitter=0.2, seed=20250220)
if a.mesh != "box":
    cells, coords, _ = mesh.download()
    mesh.close()
    rng = np.random.default_rng(1234)
    if a.mesh == "arrays":
        p = rng.permutation(coords.shape[0]).astype(np.int32)
        cells = p[cells][rng.permutation(cells.shape[0])]
        pc = np.empty_like(coords)
        pc[p] = coords
        coords = pc
    else:
        cells = np.ascontiguousarray(cells[rng.permutation(cells.shape[0])])
    mesh = af.Mesh.from_arrays(ctx, 3, cells, coords)
    del cells, coords
bsr = af.BSRFormat(mesh, 1).initialize(True)
bsr.computeSparsity()
rhs = ctx.malloc(8 * mesh.n_own_nodes)


def run():
    bsr.assemblePoissonP1(1.0, 5.5, rhs, rhs_mode="set")


times = {n: [] for n, _ in variants}
vals = {}
for r in range(a.rounds):
    for name, knobs in variants:
        for k in all_knobs:
            af.set_variant(k, knobs.get(k))
        t = time.perf_counter()
        while (time.perf_counter() - t) * 1e3 < a.settle:
            for _ in range(8):
                run()
            ctx.synchronize()
        for i in range(a.reps):
            ctx.event_record(2 * i)
            run()
            ctx.event_record(2 * i + 1)
        ctx.synchronize()
        times[name] += [ctx.event_elapsed(2 * i, 2 * i + 1) for i in range(a.reps)]
        if r == 0:
            vals[name] = (bsr.download()[2], bsr.stats()["last_kernel"])
for k in all_knobs:
    af.set_variant(k, None)
rf = bench.roofline(bsr, mesh, 1.0)
ab = rf["algorithmic_bytes_per_launch"]
kmin = rf["bytes_kernel_min"]
v0 = vals[variants[0][0]][0]
for name, _ in variants:
    t = float(np.median(times[name]))
    d = np.abs(vals[name][0] - v0).max() / np.abs(v0).max()
    print(f"{name:16s} median {t:.4f} ms  frac {ab / (t * 1e-3) / 8e12:.4f}  min-bytes frac "
          f"{kmin / (t * 1e-3) / 8e12:.4f}  kernel {vals[name][1]}  max|v - {variants[0][0]}|/max {d:.2e}  "
          f"p10 {np.percentile(times[name], 10):.4f} p90 {np.percentile(times[name], 90):.4f}", flush=True)
