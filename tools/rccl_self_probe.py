"""The RCCL data path's per-iteration cost on one GPU (AFEM_COMM_SELF=1: a
one-rank communicator runs its collectives): the C2 Poisson system's Jacobi-PCG,
fixed iterations, plain and with the one-rank RCCL communicator attached (an
empty halo: the scalars' ncclAllReduce and the exchange's bookkeeping every
iteration, no ghost data) -- what an N-rank run adds per iteration besides the
halo bytes.  usage: python tools/rccl_self_probe.py [n] [iters]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 215
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 100
ctx = af.Context(0)
mesh = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=20250220)
bsr = af.BSRFormat(mesh, 1).initialize(True)
bsr.computeSparsity()
bottom = mesh.bottom_nodes()


def system():
    ls = af.DoFLinearSystem().initialize(ctx, mesh.n_own_nodes, mesh.n_nodes)
    bsr.toLinearSystem(ls)
    bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable(), rhs_mode="set")
    ls.applyDirichletViaPenalty(bottom, 0.5, 1.0e30)
    ls.setSolverOptions(fixed_iterations=iters)
    return ls


out = {}
for mode in ("plain", "rccl_self", "plain", "rccl_self"):
    if mode == "rccl_self":
        af.set_variant("AFEM_COMM_SELF", "1")
        comm = af.Communicator(ctx, 1, 0, af.Communicator.unique_id())
    ls = system()
    if mode == "rccl_self":
        ls.set_halo(comm, [], [], [])
    st = ls.solve()
    out.setdefault(mode, []).append(st["solve_ms"] / max(1, st["iterations"]))
    print(f"{mode:10s} {st['iterations']} iterations, {st['solve_ms'] / max(1, st['iterations']):.4f} ms each, "
          f"all-reduces {st.get('n_allreduce')}, halo exchanges {st.get('n_halo')}, spmv kernel {st['spmv_kernel']}",
          flush=True)
    ls.reset()
    if mode == "rccl_self":
        af.set_variant("AFEM_COMM_SELF", None)
print({k: round(float(np.median(v)), 4) for k, v in out.items()})
