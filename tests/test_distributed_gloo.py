"""CPU, world_size 2 (and 3) over gloo: the multi-GPU decomposition logic.

Each rank builds its z-slab (owned nodes first, one ghost node/cell layer),
takes the product's halo plan (afem_structured_halo_plan, host-only C ABI:
the send / recv DoF lists libafem packs and unpacks), assembles its owned
rows (oracle), and runs the iteration the GPU path runs in ls_solve
(linear_system.hip): Jacobi preconditioner with the constraint-row flag,
x0 lifting of the constraint rows (k_cg_x0), r0 = b - A x0 after a halo
exchange, stopping reference r0.z0 over the free rows summed over ranks,
the test every `check_every` = 8 iterations, halo exchange of the search
direction before every SpMV, the two dot products summed over ranks --
with torch.distributed gloo standing in for RCCL.  The same iteration on
the GPU with more than one rank runs in tests/test_gpu_distributed.py
(host transport).  The gathered solution must match the single-domain
direct solve to 1e-10, every rank must run the same number of iterations,
and the owned rows of every slab must equal the corresponding rows of the
global matrix (owner-computes assembly needs no communication).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N, NZ = 5, 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _halo(x, plan, rank):
    nbr, sc, rc, si, ri = plan
    soff = np.concatenate([[0], np.cumsum(sc)])
    roff = np.concatenate([[0], np.cumsum(rc)])
    reqs = []
    bufs = []
    for k, q in enumerate(nbr):
        send = torch.from_numpy(x[si[soff[k]:soff[k + 1]]].copy())
        recv = torch.empty(int(rc[k]), dtype=torch.float64)
        bufs.append(recv)
        reqs.append(dist.isend(send, int(q)))
        reqs.append(dist.irecv(recv, int(q)))
    for r in reqs:
        r.wait()
    for k in range(len(nbr)):
        x[ri[roff[k]:roff[k + 1]]] = bufs[k].numpy()


def _allsum(v):
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t)
    return float(t[0])


def _worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import arcanefem_amd as af
    from oracle import oracle as O

    m = O.structured_mesh(3, N, nz=NZ, nranks=world, rank=rank)
    plan = af.structured_halo_plan(3, N, NZ, world, rank)
    n_own, n_loc = m["n_own"], m["n_local"]
    rp, cols = O.sparsity(n_loc, n_own, m["cells"])
    vals, rhs = O.assemble_poisson(n_own, m["cells"], m["coords"], rp, cols, 5.5)
    O.dirichlet_penalty(m["dirichlet"], 0.5, 1e30, rp, cols, vals, rhs)
    # distributed Jacobi-PCG: the sequence of ls_solve (linear_system.hip)
    d = np.array([vals[rp[i]:rp[i + 1]][cols[rp[i]:rp[i + 1]] == i][0] for i in range(n_own)])
    off = np.array([np.abs(vals[rp[i]:rp[i + 1]][cols[rp[i]:rp[i + 1]] != i]).sum() for i in range(n_own)])
    dinv = np.where(d != 0, 1.0 / d, 0.0)                      # k_inv_diag
    cons = np.abs(d) > 1e10 * off
    p = np.zeros(n_loc)
    x = np.where(cons, rhs * dinv, 0.0)                        # k_cg_x0
    p[:n_own] = x
    _halo(p, plan, rank)
    r = rhs - O.spmv(rp, cols, vals, p)                        # k_cg_init
    z = r * dinv
    p[:n_own] = z
    rz = _allsum(r @ z)
    rz0 = _allsum((r * z)[~cons].sum())
    if rz0 <= 0.0:
        rz0 = rz
    it, check, rtol = 0, 8, 1e-14
    converged = rz == 0.0 or np.sqrt(abs(rz / rz0)) <= rtol
    while not converged and it < 20000:
        _halo(p, plan, rank)
        q = O.spmv(rp, cols, vals, p)
        pq = _allsum(p[:n_own] @ q)
        alpha = rz / pq if pq != 0.0 else 0.0                  # k_cg_update
        x += alpha * p[:n_own]
        r -= alpha * q
        z = r * dinv
        rzn = _allsum(r @ z)
        beta = rzn / rz if rz != 0.0 else 0.0                  # k_cg_dir
        p[:n_own] = z + beta * p[:n_own]
        rz = rzn
        it += 1
        if it % check == 0:
            converged = np.sqrt(abs(rz / rz0)) <= rtol
    # owned rows vs the global matrix rows (global ids)
    l2g = m["local_to_global"]
    g = O.structured_mesh(3, N, nz=NZ)
    grp, gcols = O.sparsity(g["n_local"], g["n_own"], g["cells"])
    gvals, grhs = O.assemble_poisson(g["n_own"], g["cells"], g["coords"], grp, gcols, 5.5)
    O.dirichlet_penalty(g["dirichlet"], 0.5, 1e30, grp, gcols, gvals, grhs)
    row_err = 0.0
    for i in range(n_own):
        gi = l2g[i]
        lc = l2g[cols[rp[i]:rp[i + 1]]]
        order = np.argsort(lc)
        gseg = slice(grp[gi], grp[gi + 1])
        assert np.array_equal(lc[order], gcols[gseg])
        row_err = max(row_err, np.abs(vals[rp[i]:rp[i + 1]][order] - gvals[gseg]).max() / np.abs(gvals[gseg]).max())
    out_q.put((rank, l2g[:n_own].copy(), x, it, row_err))
    assert converged
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_pcg_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle import oracle as O

    g = O.structured_mesh(3, N, nz=NZ)
    grp, gcols = O.sparsity(g["n_local"], g["n_own"], g["cells"])
    gvals, grhs = O.assemble_poisson(g["n_own"], g["cells"], g["coords"], grp, gcols, 5.5)
    O.dirichlet_penalty(g["dirichlet"], 0.5, 1e30, grp, gcols, gvals, grhs)
    xg = np.linalg.solve(O.csr_to_dense(grp, gcols, gvals), grhs)
    x = np.full(g["n_own"], np.nan)
    its = set()
    for rank, gid, xl, it, row_err in res:
        x[gid] = xl
        its.add(it)
        assert row_err <= 1e-14
    assert len(its) == 1 and min(its) % 8 == 0
    assert not np.isnan(x).any()
    assert np.abs(x - xg).max() / np.abs(xg).max() <= 1e-10
