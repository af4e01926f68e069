"""A/B of an assembly-time environment toggle (read at every assembly) in ONE
process: one structure, the assembly timed with VAR=valA / VAR=valB
interleaved (HIP events, median).
usage: python tools/ab_asm_env.py VAR valA valB [n] [reps] [k]   (k = 3: block-3 elasticity, C3)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402

var, va, vb = sys.argv[1], sys.argv[2], sys.argv[3]
n = int(sys.argv[4]) if len(sys.argv) > 4 else 215
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 20
k = int(sys.argv[6]) if len(sys.argv) > 6 else 1
ctx = af.Context(0)
mesh = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=20250220)
bsr = af.BSRFormat(mesh, k).initialize(True)
bsr.computeSparsity()
ls = af.DoFLinearSystem().initialize(ctx, k * mesh.n_own_nodes)
vals = {}
times = {va: [], vb: []}
for r in range(reps):
    for v in (va, vb):
        af.set_variant(var, v)  # the library caches the environment at its first read
        ctx.event_record(0)
        if k == 1:
            bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable(), rhs_mode="set")
        else:
            bsr.assembleElasticityP1Ex(1.0e5, 1.5e5, 0.0, (0.0, 0.0, -1.0), ls.rhsVariable(), rhs_mode="set")
        ctx.event_record(1)
        ctx.synchronize()
        if r >= 2:
            times[v].append(ctx.event_elapsed(0, 1))
        if r == reps - 1:
            vals[v] = bsr.download()[2]
print("bitwise equal:", np.array_equal(vals[va], vals[vb]),
      "max |diff| / max |value|: %.3e" % (np.abs(vals[va] - vals[vb]).max() / np.abs(vals[va]).max()), flush=True)
for v in times:
    print(f"{var}={v}: median {np.median(times[v]):.4f} ms  min {np.min(times[v]):.4f}", flush=True)
