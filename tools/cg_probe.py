"""A/B of CG variants in ONE process: C2 Poisson system, fixed Jacobi-PCG
iterations, device time per iteration (solve_ms of the ABI's stats), for each
value of an environment toggle read at solve time.
usage: python tools/cg_probe.py VAR val1 [val2 ...] [--n 215] [--iters 50] [--reps 3]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("var")
ap.add_argument("vals", nargs="+")
ap.add_argument("--n", type=int, default=215)
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
ctx = af.Context(0)
mesh = af.Mesh.structured(ctx, 3, a.n, jitter=0.2, seed=20250220)
bsr = af.BSRFormat(mesh, 1).initialize(True)
bsr.computeSparsity()
ls = af.DoFLinearSystem().initialize(ctx, mesh.n_own_nodes, mesh.n_nodes)
bsr.toLinearSystem(ls)
bottom = mesh.bottom_nodes()
db = ctx.malloc(4 * bottom.size)
ctx.to_device(db, bottom)
bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable(), rhs_mode="set")
ls.applyDirichletViaPenaltyDevice(db, bottom.size, 0.5, 1.0e30)
ls.applyBoundaryConditions()
ls.setSolverOptions(fixed_iterations=a.iters)
res = {v: [] for v in a.vals}
sols = {}
for r in range(a.reps + 1):
    for v in a.vals:
        af.set_variant(a.var, v)  # the library caches the environment at its first read
        st = ls.solve()
        if r:
            res[v].append(st["solve_ms"] / a.iters)
        sols[v] = (ctx.to_host(ls.solutionVariable(), mesh.n_own_nodes, np.float64), st["rel_residual"])
ref = sols[a.vals[0]][0]
for v in a.vals:
    d = np.max(np.abs(sols[v][0] - ref)) / max(np.max(np.abs(ref)), 1e-300)
    print(f"{a.var}={v}: {np.median(res[v]):.4f} ms/iter  rel_res {sols[v][1]:.3e}  max rel diff vs first {d:.2e}",
          flush=True)
