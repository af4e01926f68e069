"""A/B of the cell-first cube kernel against the row-strip kernels on one
generator box in one process (AFEM_ASSEMBLY_CUBES toggled per call,
interleaved, HIP events), the values compared.
usage: python tools/cubes_ab.py [n] [reps] [zs ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 215
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
zss = sys.argv[3:] or ["16"]
ctx = af.Context(0)
mesh = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=20250220)
bsr = af.BSRFormat(mesh, 1).initialize(True)
bsr.computeSparsity()
rhs = ctx.malloc(8 * mesh.n_own_nodes)
modes = [("strip", "0", None)] + [(f"cubes zs={z}", "1", z) for z in zss]
times = {m: [] for m, _, _ in modes}
vals = {}
for r in range(reps + 2):
    for name, cubes, zs in modes:
        af.set_variant("AFEM_ASSEMBLY_CUBES", cubes)
        af.set_variant("AFEM_CUBES_ZS", zs)
        ctx.event_record(0)
        bsr.assemblePoissonP1(1.0, 5.5, rhs, rhs_mode="set")
        ctx.event_record(1)
        ctx.synchronize()
        if r >= 2:
            times[name].append(ctx.event_elapsed(0, 1))
        if r == reps + 1:
            vals[name] = bsr.download()[2]
rf = bench.roofline(bsr, mesh, 1.0)
ab = rf["algorithmic_bytes_per_launch"]
for name, _, _ in modes:
    t = float(np.median(times[name]))
    d = np.abs(vals[name] - vals["strip"]).max() / np.abs(vals["strip"]).max()
    print(f"{name:14s} median {t:.4f} ms  frac {ab / (t * 1e-3) / 8e12:.4f}  max|v - strip|/max {d:.2e}  "
          f"all {' '.join(f'{x:.3f}' for x in times[name])}", flush=True)
