"""A/B on C2 handed over as arrays in a random numbering (bench.py's c2_arrays
input: seed 1234) in ONE process: one structure per variant of a library knob
(e.g. AFEM_CANON 1 / 0; the knob stays set for that variant's assemblies too),
assembly kernels timed interleaved (HIP events,
median of `reps`), values compared between the variants.
usage: python tools/arrays_ab.py VAR valA valB [n] [reps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402

var, va, vb = sys.argv[1], sys.argv[2], sys.argv[3]
n = int(sys.argv[4]) if len(sys.argv) > 4 else 215
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 10
ctx = af.Context(0)
m0 = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=20250220)
cells, coords, _ = m0.download()
m0.close()
rng = np.random.default_rng(1234)
p = rng.permutation(coords.shape[0]).astype(np.int32)
cells = p[cells][rng.permutation(cells.shape[0])]
pc = np.empty_like(coords)
pc[p] = coords
mesh = af.Mesh.from_arrays(ctx, 3, cells, pc)
del cells, coords, pc
rhs = ctx.malloc(8 * mesh.n_own_nodes)
variants = []
for v in (va, vb):
    af.set_variant(var, v)
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    bsr.computeSparsity()
    st = bsr.stats()
    print(v, {k: st[k] for k in ("n_slices", "uniform_slices", "stencil_slices", "general_slices", "brick_order",
                                 "max_slice_nodes")}, flush=True)
    variants.append((v, bsr))
times = {v: [] for v, _ in variants}
for r in range(reps + 2):
    for v, bsr in variants:
        af.set_variant(var, v)  # knobs read at assembly time (AFEM_ASSEMBLY_CUBES) as well as at the build
        ctx.event_record(0)
        bsr.assemblePoissonP1(1.0, 5.5, rhs, rhs_mode="set")
        ctx.event_record(1)
        ctx.synchronize()
        if r >= 2:
            times[v].append(ctx.event_elapsed(0, 1))
af.set_variant(var, None)
vals = [bsr.download()[2] for _, bsr in variants]
for v, _ in variants:
    print(f"{var}={v}: median {np.median(times[v]):.4f} ms  all {' '.join(f'{t:.3f}' for t in times[v])}", flush=True)
print(f"max |a - b| / max |a| = {np.abs(vals[0] - vals[1]).max() / np.abs(vals[0]).max():.2e}")
