"""AMG probe: the unstructured leg's system (L-shape-3D refined
`levels` times, Poisson, z-min nodes clamped by penalty) solved by the AMG-PCG
for each variant (comma list of AFEM_AMG_* = value, '-' = defaults), with the
level sizes (AFEM_AMG_VERBOSE) on stderr; Jacobi once for reference.
usage: python tools/amg_probe.py levels rtol variant [variant ...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402
from arcanefem_amd.gmsh import read_gmsh  # noqa: E402
from bench import refine_tets  # noqa: E402

levels, rtol = int(sys.argv[1]), float(sys.argv[2])
ctx = af.Context(0)
gm = read_gmsh(os.path.join(ROOT, "tests", "golden", "L-shape-3D.msh"))
cells, coords = refine_tets(gm.cells, gm.coords, levels, "cpu")
mesh = af.Mesh.from_arrays(ctx, 3, cells, coords)
z = coords[:, 2]
dn = np.nonzero(z <= z.min() + 1e-9 * max(1.0, abs(z.min())))[0].astype(np.int32)
del cells, coords, z
bsr = af.BSRFormat(mesh, 1).initialize(True)
bsr.computeSparsity()
ls = af.DoFLinearSystem().initialize(ctx, mesh.n_own_nodes, mesh.n_nodes)
bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable())
bsr.toLinearSystem(ls)
print(f"{mesh.n_own_nodes} rows", flush=True)
ref = None
for spec in ["jacobi"] + sys.argv[3:]:
    kv = [] if spec in ("-", "jacobi") else [x.split("=") for x in spec.split(",")]
    for k, v in kv:
        af.set_variant(k, v)
    if not any(k == "AFEM_AMG_VERBOSE" for k, _ in kv):
        af.set_variant("AFEM_AMG_VERBOSE", "1")  # (=2 in a variant: each independent-set round too)
    ls.applyDirichletViaPenalty(dn, 0.5, 1.0e30)
    ls.setSolverOptions(rtol=rtol, max_iter=100000, method="pcg", preconditioner="jacobi" if spec == "jacobi" else "amg")
    t0 = time.perf_counter()
    st = ls.solve()
    wall = (time.perf_counter() - t0) * 1e3
    x = ls.solution_host().copy()
    if ref is None:
        ref = x
    d = np.abs(x - ref).max() / np.abs(ref).max()
    print(f"{spec:40s} it {st['iterations']:5d} solve {st['solve_ms']:8.1f} ms (setup {st['amg_setup_ms']:6.1f}) "
          f"levels {st['amg_levels']} coarsest {st['amg_coarse_rows']} complexity {st['amg_complexity']:.3f} "
          f"per-it {(st['solve_ms'] - st['amg_setup_ms']) / max(1, st['iterations']):.3f} ms diff {d:.1e}",
          flush=True)
    for k, _ in kv:
        af.set_variant(k, None)
