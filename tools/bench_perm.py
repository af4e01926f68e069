"""Assembly time on the C2 box with a seeded random node/cell numbering (the
SURVEY §8d robustness variant: an unstructured-like numbering, node-order
slices, no bricks).  usage: python tools/bench_perm.py [n] [reps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402
from oracle import oracle as O  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 215
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
t0 = time.time()
ref = O.structured_mesh(3, n, jitter=0.2, seed=20250220)
rng = np.random.default_rng(1234)
nn = ref["n_local"]
p = rng.permutation(nn).astype(np.int64)
cells = p[ref["cells"]].astype(np.int32)[rng.permutation(ref["cells"].shape[0])]
coords = np.empty_like(ref["coords"])
coords[p] = ref["coords"]
print(f"mesh n={n}: {nn} nodes, {cells.shape[0]} cells, host prep {time.time() - t0:.1f} s", flush=True)
ctx = af.Context(0)
mesh = af.Mesh.from_arrays(ctx, 3, cells, coords)
bsr = af.BSRFormat(mesh, 1).initialize(True)
t0 = time.time()
bsr.computeSparsity()
ctx.synchronize()
print(f"sparsity {1e3 * (time.time() - t0):.1f} ms; stats {bsr.stats()}", flush=True)
ls = af.DoFLinearSystem().initialize(ctx, mesh.n_own_nodes, mesh.n_nodes)
for _ in range(2):
    bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable(), rhs_mode="set")
ctx.synchronize()
for i in range(reps):
    ctx.event_record(2 * i)
    bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable(), rhs_mode="set")
    ctx.event_record(2 * i + 1)
ctx.synchronize()
ms = float(np.mean([ctx.event_elapsed(2 * i, 2 * i + 1) for i in range(reps)]))
print(f"assembly {ms:.3f} ms = {nn / ms / 1e3:.1f} MDoF/s (random numbering)", flush=True)
