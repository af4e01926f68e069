"""A/B of a structure-build environment toggle in ONE process (same box, same
clock): builds the Poisson structure of a Kuhn box once per variant and times
the assembly kernels (HIP events, median of `reps`) interleaved.
usage: python tools/ab_env.py VAR valA valB [n] [reps] [valC ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402

var, va, vb = sys.argv[1], sys.argv[2], sys.argv[3]
n = int(sys.argv[4]) if len(sys.argv) > 4 else 215
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 20
extra = sys.argv[6:]  # more values (each its own structure, built in this order)
ctx = af.Context(0)
mesh = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=20250220)
variants = []
for v in [va, vb] + extra:
    af.set_variant(var, v)  # the library caches the environment at its first read
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    bsr.computeSparsity()
    ls = af.DoFLinearSystem().initialize(ctx, mesh.n_own_nodes)
    variants.append((v, bsr, ls))
    print(v, bsr.stats(), flush=True)
times = {v: [] for v, _, _ in variants}
for r in range(reps):
    for i, (v, bsr, ls) in enumerate(variants[::-1] if os.environ.get("AB_REVERSE") else variants):
        ctx.event_record(0)
        bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable(), rhs_mode="set")
        ctx.event_record(1)
        ctx.synchronize()
        if r >= 2:
            times[v].append(ctx.event_elapsed(0, 1))
_, _, va_vals = variants[0][1].download()
_, _, vb_vals = variants[1][1].download()
print("bitwise equal:", np.array_equal(va_vals, vb_vals))
for v in times:
    print(f"{var}={v}: median {np.median(times[v]):.4f} ms  min {np.min(times[v]):.4f}", flush=True)
