"""A/B of the cell-unit kernel's plan knobs at the C2 size in one process:
for each variant (comma list of KEY=VALUE, '-' = defaults) a fresh structure
and plan, then the kernel time (median of `reps`, HIP events) with the Poisson
module's element (elements::PoissonTet4) and the lean cofactor element.
Variant keys UN=k (k = 1..4, 6, 8) and PAD=p (-1: XOR-swizzled rows) run the kernel with k functor
evaluations in flight per lane and LDS planes of rows + p (gx_assemble_unrolled;
defaults: the header's, 4 and 0).
usage: python tools/generic_ab.py n reps variant [variant ...]
n = "lshape<k>": the unstructured leg's mesh instead (L-shape-3D refined k times, slice-piece units;
the functor library loaded before the refinement imports torch, bench.py c2_generic_leg)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "examples"))
import arcanefem_amd as af  # noqa: E402
import generic_example as gx  # noqa: E402

reps = int(sys.argv[2])
ctx = af.Context(0)
gx.load()
if sys.argv[1].startswith("lshape"):
    import bench
    from arcanefem_amd.gmsh import read_gmsh

    gm = read_gmsh(os.path.join(ROOT, "tests", "golden", "L-shape-3D.msh"))
    cells, coords = bench.refine_tets(gm.cells, gm.coords, int(sys.argv[1][6:]), "cpu")
    mesh = af.Mesh.from_arrays(ctx, 3, cells, coords)
    del cells, coords
else:
    mesh = af.Mesh.structured(ctx, 3, int(sys.argv[1]), jitter=0.2, seed=20250220)
ref = None
first = None
for spec in sys.argv[3:]:
    kv = [] if spec == "-" else [x.split("=") for x in spec.split(",")]
    un = [int(v) for k, v in kv if k == "UN"]
    pad = [int(v) for k, v in kv if k == "PAD"]
    kv = [(k, v) for k, v in kv if k not in ("UN", "PAD")]

    def run(kind):
        if un or pad:
            gx.assemble_unrolled(bsr, kind, un[0] if un else 4, overwrite=True, pad=pad[0] if pad else 0)
        else:
            gx.assemble(bsr, kind, gx.UNITS, overwrite=True)
    for k, v in kv:
        af.set_variant(k, v)
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    bsr.computeSparsity()
    plan = bsr.functor_plan()
    st = bsr.stats()
    nnz = bsr.view().nnz_blocks
    ab = 4 * st["n_incidences"] + 24 * mesh.n_nodes + 8 * (mesh.n_own_nodes + 1) + 12 * nnz
    out = []
    for kind in (gx.POISSON, gx.POISSON_LEAN):
        run(kind)
        ctx.synchronize()
        for i in range(reps):
            ctx.event_record(2 * i)
            run(kind)
            ctx.event_record(2 * i + 1)
        ctx.synchronize()
        t = float(np.median([ctx.event_elapsed(2 * i, 2 * i + 1) for i in range(reps)]))
        out.append(f"{t:.3f} ms ({ab / (t * 1e-3) / 8e12:.3f})")
    v = bsr.download()[2]
    if ref is None:
        bsr.assemblePoissonP1(1.0, 0.0)
        ref = bsr.download()[2]
    err = float(np.abs(v - ref).max() / np.abs(ref).max())
    if first is None:
        first = v
    err = f"{err:.1e} bits-as-first {np.array_equal(v, first)}"
    print(f"{spec:40s} units {plan['n_units']:6d} rl {plan['rows_per_layer']:2d} evals/cell "
          f"{plan['n_entries'] / mesh.n_cells:.3f} packed {plan['packed']} patterns {plan['n_patterns']} | module {out[0]} | "
          f"lean {out[1]} | err {err}", flush=True)
    for k, _ in kv:
        af.set_variant(k, None)
    bsr.close()
