"""Multigrid-preconditioned PCG against point Jacobi on structured boxes
(Poisson k=1, elasticity k=3): iterations, time, solution difference.
usage: python tools/mg_probe.py [n ...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402

ns = [int(a) for a in sys.argv[1:]] or [32]
pcs = os.environ.get("MG_PCS", "jacobi,multigrid").split(",")
ctx = af.Context(0)
for n in ns:
    for k in (1, 3):
        mesh = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=20250220)
        bsr = af.BSRFormat(mesh, k).initialize(True)
        bsr.computeSparsity()
        ls = af.DoFLinearSystem().initialize(ctx, k * mesh.n_own_nodes)
        if k == 1:
            bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable(), rhs_mode="set")
        else:
            bsr.assembleElasticityP1Ex(1.2e6, 1.6e6, 4e6, (0.0, 0.0, -1.0), ls.rhsVariable(), rhs_mode="set")
        bsr.toLinearSystem(ls)
        fixed = np.arange((n + 1) ** 2, dtype=np.int32)  # the z = 0 node layer
        dofs = (k * fixed[:, None] + np.arange(k)[None, :]).ravel().astype(np.int32)
        ls.applyDirichletViaPenalty(dofs, 0.5, 1e30)
        res = {}
        for pc in pcs:
            ls.setSolverOptions(rtol=1e-10, preconditioner=pc, max_iter=20000)
            t0 = time.perf_counter()
            st = ls.solve()
            ctx.synchronize()
            t = time.perf_counter() - t0
            res[pc] = ls.solution_host().copy()
            print(f"k={k} n={n} {pc:10s} it {st['iterations']:6d} conv {st['converged']} rel {st['rel_residual']:.2e} "
                  f"{t * 1e3:8.1f} ms", flush=True)
        if len(res) == 2:
            a, b = list(res.values())
            print(f"  max |diff| / max |x| = {np.abs(a - b).max() / np.abs(a).max():.2e}", flush=True)
        ls.reset()
        bsr.close()
        mesh.close()
