"""CPU, world_size 2 (and 3) over gloo: the multi-GPU decomposition logic.

Each rank builds its z-slab (owned nodes first, one ghost node/cell layer),
takes the product's halo plan (afem_structured_halo_plan, host-only C ABI),
assembles its owned rows (oracle), and runs the same distributed Jacobi-PCG
the GPU path runs (halo exchange of the search direction before every SpMV,
sum-all-reduce of the two dot products, constraint rows excluded from the
stopping reference) with torch.distributed gloo standing in for RCCL.  The
gathered solution must match the single-domain direct solve to 1e-10, and the
owned rows of every slab must equal the corresponding rows of the global
matrix (owner-computes assembly needs no communication).
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
    # distributed Jacobi-PCG (ls_solve in linear_system.hip)
    d = np.array([vals[rp[i]:rp[i + 1]][cols[rp[i]:rp[i + 1]] == i][0] for i in range(n_own)])
    off = np.array([np.abs(vals[rp[i]:rp[i + 1]][cols[rp[i]:rp[i + 1]] != i]).sum() for i in range(n_own)])
    dinv = 1.0 / d
    cons = np.abs(d) > 1e10 * off
    x = np.zeros(n_own)
    r = rhs.copy()
    z = r * dinv
    p = np.zeros(n_loc)
    p[:n_own] = z
    rz = _allsum(r @ z)
    rz0 = _allsum((r * z)[~cons].sum())
    it = 0
    while it < 5000 and np.sqrt(abs(rz / rz0)) > 1e-15:
        _halo(p, plan, rank)
        q = O.spmv(rp, cols, vals, p)
        alpha = rz / _allsum(p[:n_own] @ q)
        x += alpha * p[:n_own]
        r -= alpha * q
        z = r * dinv
        rzn = _allsum(r @ z)
        p[:n_own] = z + (rzn / rz) * p[:n_own]
        rz = rzn
        it += 1
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
    for rank, gid, xl, it, row_err in res:
        x[gid] = xl
        assert row_err <= 1e-14
    assert not np.isnan(x).any()
    assert np.abs(x - xg).max() / np.abs(xg).max() <= 1e-10
