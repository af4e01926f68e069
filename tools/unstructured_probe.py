"""Unstructured-mesh legs (the reference's L-shape-3D Gmsh mesh refined
`levels` times, Hilbert-ordered slices): bench.unstructured_leg (Poisson) and,
with --elasticity, the block-3 assembly on the same mesh.
usage: python tools/unstructured_probe.py [levels] [--elasticity]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402
import bench  # noqa: E402

levels = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else 6
ctx = af.Context(0)
print(json.dumps(bench.unstructured_leg(ctx, af, "L-shape-3D.msh", levels)), flush=True)
if "--elasticity" in sys.argv:
    from arcanefem_amd.gmsh import read_gmsh

    gm = read_gmsh(os.path.join(ROOT, "tests", "golden", "L-shape-3D.msh"))
    cells, coords = bench.refine_tets(gm.cells, gm.coords, levels - 1, "cpu")
    mesh = af.Mesh.from_arrays(ctx, 3, cells, coords)
    bsr = af.BSRFormat(mesh, 3).initialize(False)
    bsr.computeSparsity()
    rhs = ctx.malloc(8 * 3 * mesh.n_own_nodes)
    ts = []
    for i in range(7):
        ctx.event_record(250)
        bsr.assembleElasticityP1Ex(1.0e5, 1.5e5, 0.0, (0.0, 0.0, -1.0), rhs, rhs_mode="set")
        ctx.event_record(251)
        ctx.synchronize()
        if i >= 2:
            ts.append(ctx.event_elapsed(250, 251))
    st = bsr.stats()
    nnz_b = bsr.view().nnz_blocks
    n_own = mesh.n_own_nodes
    ab = 4 * int(st["n_incidences"]) + 24 * mesh.n_nodes + 8 * (n_own + 1) + 76 * nnz_b + 24 * n_own
    kms = float(np.median(ts))
    print(json.dumps({"elasticity_levels": levels - 1, "nodes": n_own, "tets": mesh.n_cells, "kernel_ms": kms,
                      "frac": ab / (kms * 1e-3) / 8e12, "last_kernel": int(st["last_kernel"]),
                      "max_slice_width": int(st["max_slice_width"])}), flush=True)
