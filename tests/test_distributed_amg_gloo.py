"""CPU, world_size 2 and 3 over gloo: the decomposition logic of the
distributed algebraic multigrid (arcanefem_amd/csrc/amg.hip, round 6).

Each rank takes its z-slab (owned nodes first, one ghost layer) and the
product's halo plan (afem_structured_halo_plan, host-only C ABI), assembles its
owned rows (oracle), aggregates its own rows with a ghost-blind local rule, and
then mirrors in numpy what amg.hip does with them:
  * ghost_aggregates: the owners' aggregate ids exchanged through the fine
    halo;
  * build_dist_coarse: the coarse ghost columns numbered neighbour by
    neighbour in increasing owner aggregate id, the coarse send list to rank s
    = the sorted aggregates of the rows sent to s, A_c = P^T A P keyed through
    the column map;
  * build_gathered: this rank's coarse rows in the global numbering
    (aggregates numbered rank by rank).
Checked: every rank's coarse send list to s equals, entry by entry, what s
expects to receive (its coarse ghosts from this rank, owner ids); a coarse
halo exchange fills every coarse ghost with its owner's value; the
distributed coarse operator gathered over the ranks and the gathered-level
COO both equal P^T A P of the global matrix with the union of the aggregates
(torch.distributed gloo stands in for RCCL / the host transport).  The same
construction runs on the GPU in tests/test_gpu_distributed.py
(test_distributed_amg_subdomains: 1 / 2 / 4 / 8 ranks against the oracle) and
through RCCL on one GPU (test_rccl_self_loop_solve).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N, NZ = 5, 9


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _exchange(x, nbr, sl, rl):
    """halo_exchange: x[recv ids of q] = the neighbour's x[its send ids to me]."""
    reqs, bufs = [], []
    for k, q in enumerate(nbr):
        send = torch.from_numpy(np.ascontiguousarray(x[sl[k]], dtype=np.float64))
        recv = torch.empty(len(rl[k]), dtype=torch.float64)
        bufs.append(recv)
        reqs.append(dist.isend(send, int(q)))
        reqs.append(dist.irecv(recv, int(q)))
    for r in reqs:
        r.wait()
    for k in range(len(nbr)):
        x[rl[k]] = bufs[k].numpy()


def _lists(x, nbr):
    """Send one integer list to each neighbour, receive one from each."""
    out = []
    for k, q in enumerate(nbr):
        n_me = torch.tensor([len(x[k])], dtype=torch.int64)
        n_it = torch.empty(1, dtype=torch.int64)
        a, b = dist.isend(n_me, int(q)), dist.irecv(n_it, int(q))
        a.wait()
        b.wait()
        send = torch.tensor(np.asarray(x[k], dtype=np.int64))
        recv = torch.empty(int(n_it[0]), dtype=torch.int64)
        reqs = [dist.isend(send, int(q))] if len(x[k]) else []
        if int(n_it[0]):
            reqs.append(dist.irecv(recv, int(q)))
        for r in reqs:
            r.wait()
        out.append(recv.numpy())
    return out


def _aggregate(n, rp, cols):
    """A deterministic ghost-blind aggregation of the owned rows: in row order,
    an unassigned row starts an aggregate with its unassigned owned neighbours
    (the shape differs from amg.hip's MIS; the coarse construction does not
    depend on how the aggregates were found)."""
    agg = np.full(n, -1, dtype=np.int64)
    k = 0
    for i in range(n):
        if agg[i] >= 0:
            continue
        agg[i] = k
        for j in cols[rp[i]:rp[i + 1]]:
            if j < n and agg[j] < 0:
                agg[j] = k
        k += 1
    return agg, k


def _galerkin(n, rp, cols, vals, agg, cmap, nrow):
    """Sum of a_ij over (agg i, cmap j), ghost-aware: a dict of the coarse entries."""
    out = {}
    for i in range(n):
        for k in range(rp[i], rp[i + 1]):
            c = cmap[cols[k]]
            if c < 0:
                continue
            key = (int(agg[i]), int(c))
            out[key] = out.get(key, 0.0) + vals[k]
    return out


def _worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import arcanefem_amd as af
    from oracle import oracle as O

    m = O.structured_mesh(3, N, nz=NZ, nranks=world, rank=rank)
    nbr, sc, rc, si, ri = af.structured_halo_plan(3, N, NZ, world, rank)
    soff = np.concatenate([[0], np.cumsum(sc)])
    roff = np.concatenate([[0], np.cumsum(rc)])
    sl = [si[soff[k]:soff[k + 1]] for k in range(len(nbr))]
    rl = [ri[roff[k]:roff[k + 1]] for k in range(len(nbr))]
    n_own, n_loc = m["n_own"], m["n_local"]
    rp, cols = O.sparsity(n_loc, n_own, m["cells"])
    vals, _ = O.assemble_poisson(n_own, m["cells"], m["coords"], rp, cols, 5.5)
    agg, nc = _aggregate(n_own, rp, cols)
    # ghost_aggregates: the owners' ids through the fine halo, the owner ranks from the receive lists
    gv = np.zeros(n_loc)
    gv[:n_own] = agg
    _exchange(gv, nbr, sl, rl)
    gown = np.full(n_loc, -1, dtype=np.int64)
    for k, q in enumerate(nbr):
        gown[rl[k]] = q
    gagg = gv.astype(np.int64)
    # build_dist_coarse: coarse ghosts neighbour by neighbour, increasing owner id
    cmap = np.full(n_loc, -1, dtype=np.int64)
    cmap[:n_own] = agg
    nxt = nc
    csend, crecv, cexpect = [], [], []
    cghost_owner = {}
    for k, q in enumerate(nbr):
        s = np.unique(agg[sl[k]])
        csend.append(s)
        r = np.unique(gagg[rl[k]])
        cexpect.append(r)
        crecv.append(np.arange(nxt, nxt + r.size))
        for j in rl[k]:
            cmap[j] = nxt + int(np.searchsorted(r, gagg[j]))
        for t, a in enumerate(r):
            cghost_owner[nxt + t] = (int(q), int(a))
        nxt += r.size
    # every rank's coarse send list to s is, entry by entry, what s expects from it
    got = _lists(csend, nbr)
    for k in range(len(nbr)):
        assert np.array_equal(got[k], cexpect[k]), (rank, nbr[k])
    # offsets of the gathered numbering (aggregates numbered rank by rank)
    cnt = torch.zeros(world, dtype=torch.float64)
    cnt[rank] = nc
    dist.all_reduce(cnt)
    off = np.concatenate([[0], np.cumsum(cnt.numpy().astype(np.int64))])
    # a coarse halo exchange: ghosts receive their owners' global ids
    cv = np.zeros(nxt)
    cv[:nc] = off[rank] + np.arange(nc)
    _exchange(cv, nbr, csend, crecv)
    for c in range(nc, nxt):
        q, a = cghost_owner[c]
        assert cv[c] == off[q] + a
    # the distributed coarse operator, its columns to global ids
    Ac = _galerkin(n_own, rp, cols, vals, agg, cmap, nc)
    glob = {}
    for (i, c), v in Ac.items():
        gc = off[rank] + c if c < nc else off[cghost_owner[c][0]] + cghost_owner[c][1]
        glob[(int(off[rank] + i), int(gc))] = v
    # build_gathered's COO: the global column map directly
    gmap = np.full(n_loc, -1, dtype=np.int64)
    gmap[:n_own] = off[rank] + agg
    for j in range(n_own, n_loc):
        if gown[j] >= 0:
            gmap[j] = off[gown[j]] + gagg[j]
    Ag = _galerkin(n_own, rp, cols, vals, agg, gmap, nc)
    Ag = {(int(off[rank] + i), int(c)): v for (i, c), v in Ag.items()}
    l2g = m["local_to_global"]
    out_q.put((rank, l2g[:n_own].copy(), (off[rank] + agg).copy(), glob, Ag))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_amg_coarse_levels_gloo(world):
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
    gvals, _ = O.assemble_poisson(g["n_own"], g["cells"], g["coords"], grp, gcols, 5.5)
    gagg = np.full(g["n_own"], -1, dtype=np.int64)
    dist_op, gath_op = {}, {}
    for rank, gid, aggs, glob, Ag in res:
        gagg[gid] = aggs
        dist_op.update(glob)
        gath_op.update(Ag)
    assert (gagg >= 0).all()
    ref = _galerkin(g["n_own"], grp, gcols, gvals, gagg, gagg, int(gagg.max()) + 1)
    assert set(ref) == set(dist_op) == set(gath_op)
    scale = max(abs(v) for v in ref.values())
    for k, v in ref.items():
        assert abs(dist_op[k] - v) <= 1e-13 * scale and abs(gath_op[k] - v) <= 1e-13 * scale
