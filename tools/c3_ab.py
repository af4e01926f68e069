"""A/B of assembly knobs on the C3 leg (block-3 elasticity, Kuhn box n), one
process, settled clocks, rotating rounds like tools/ab_knobs.py: each
variant's median and its values' largest difference from the first variant's.
usage: python tools/c3_ab.py [--n 170] 'A: KNOB=v' 'B: KNOB=w' ..."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=170)
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--settle", type=float, default=100.0)
ap.add_argument("variants", nargs="+")
a = ap.parse_args()
variants = []
for v in a.variants:
    name, _, kv = v.partition(":")
    variants.append((name.strip(), dict(x.strip().split("=") for x in kv.split(",") if "=" in x)))
all_knobs = sorted({k for _, kn in variants for k in kn})
E, nu = 21.0e5, 0.28
lam, mu2 = E * nu / ((1 + nu) * (1 - 2 * nu)), E / (1 + nu)
ctx = af.Context(0)
mesh = af.Mesh.structured(ctx, 3, a.n, jitter=0.2, seed=20250220)
bsr = af.BSRFormat(mesh, 3).initialize(False)
bsr.computeSparsity()
rhs = ctx.malloc(8 * 3 * mesh.n_own_nodes)
times = {n: [] for n, _ in variants}
first, diffs = None, {}
for rnd in range(a.rounds):
    for name, knobs in variants:
        for k in all_knobs:
            af.set_variant(k, knobs.get(k))
        fn = lambda: bsr.assembleElasticityP1Ex(lam, mu2, 0.0, (0.0, 0.0, -1.0), rhs, rhs_mode="set")  # noqa: E731
        ks, _ = bench.time_launches(ctx, fn, a.reps, 2, a.settle)
        times[name] += ks
        if rnd == 0:
            v = bsr.download()[2]
            if first is None:
                first = v
            diffs[name] = float(np.abs(v - first).max() / np.abs(first).max())
for k in all_knobs:
    af.set_variant(k, None)
for name, _ in variants:
    t = np.array(times[name])
    print(f"{name:16s} median {np.median(t):.4f} ms  p10 {np.percentile(t, 10):.4f} p90 {np.percentile(t, 90):.4f}"
          f"  max|v - first|/max {diffs[name]:.2e}", flush=True)
