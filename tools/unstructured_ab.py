"""A/B of assembly knobs on the unstructured leg's mesh (L-shape-3D refined
`--levels` times), one process, settled clocks, rotating rounds like
tools/ab_knobs.py: each variant's median and its values' largest difference
from the first variant's (0 = bitwise equal).
usage: python tools/unstructured_ab.py [--levels 6] 'A: KNOB=v' 'B: KNOB=w' ..."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402
import bench  # noqa: E402
from arcanefem_amd.gmsh import read_gmsh  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--levels", type=int, default=6)
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

ctx = af.Context(0)
gm = read_gmsh(os.path.join(ROOT, "tests", "golden", "L-shape-3D.msh"))
cells, coords = bench.refine_tets(gm.cells, gm.coords, a.levels, "cpu")
mesh = af.Mesh.from_arrays(ctx, 3, cells, coords)
del cells, coords
bsr = af.BSRFormat(mesh, 1).initialize(True)
bsr.computeSparsity()
print({k: v for k, v in bsr.stats().items() if "slice" in k}, flush=True)
rhs = ctx.malloc(8 * mesh.n_own_nodes)
times = {n: [] for n, _ in variants}
first = None
diffs = {}
for rnd in range(a.rounds):
    for name, knobs in variants:
        for k in all_knobs:
            af.set_variant(k, knobs.get(k))
        fn = lambda: bsr.assemblePoissonP1(1.0, 5.5, rhs, rhs_mode="set")  # noqa: E731
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
