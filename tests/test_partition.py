"""CPU: libafem's node partitioner and subdomain plans (host C++ behind the C
ABI: afem_partition_rcb, afem_subdomain_plan) on the reference Gmsh meshes.

The plan restates what Arcane's ghost layer + femutils/FemDoFsOnNodes.cc:71-128
(computeSynchronizeInfos) give the FEM module; the properties checked here are
the ones the distributed assembly and CG rely on:
- the owned nodes of the ranks tile the mesh, sizes balanced by the RCB;
- every cell with an owned node is local, and its nodes are local (the owned
  rows are complete: the row-owned assembly needs no exchange);
- the ghosts are exactly the non-owned nodes of the local cells;
- rank r's send list to s is rank s's receive list from r, entry by entry
  (global ids), and each receive list holds ghosts owned by the sender;
- a distributed SpMV (owned rows of the local matrices, ghost values taken
  from the owners through the lists) equals the global SpMV.
"""
import os

import numpy as np
import pytest

import arcanefem_amd as af
from arcanefem_amd.gmsh import read_gmsh
from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
MESHES = ["sphere_cut.msh", "L-shape-3D.msh", "L-shape.msh", "circle_cut.msh"]


def _mesh(name):
    return read_gmsh(os.path.join(HERE, "golden", name))


@pytest.mark.parametrize("name", MESHES)
@pytest.mark.parametrize("nparts", [1, 2, 3, 4, 7])
def test_rcb_partition_tiles_and_balances(name, nparts):
    gm = _mesh(name)
    part = af.partition_rcb(gm.dim, gm.coords, nparts)
    assert part.shape == (gm.n_nodes,)
    assert part.min() >= 0 and part.max() < nparts
    cnt = np.bincount(part, minlength=nparts)
    ideal = gm.n_nodes / nparts
    assert cnt.min() > 0
    assert cnt.max() - cnt.min() <= nparts  # proportional splits, rounded per level
    assert abs(cnt.max() - ideal) <= nparts
    # deterministic
    assert np.array_equal(part, af.partition_rcb(gm.dim, gm.coords, nparts))


@pytest.mark.parametrize("name", MESHES)
@pytest.mark.parametrize("nparts", [2, 3, 5])
def test_subdomain_plans_are_consistent(name, nparts):
    gm = _mesh(name)
    part = af.partition_rcb(gm.dim, gm.coords, nparts)
    plans = [af.subdomain_plan(gm.cells, part, nparts, r) for r in range(nparts)]
    owned_all = np.concatenate([p["local_to_global"][:p["n_own"]] for p in plans])
    assert np.array_equal(np.sort(owned_all), np.arange(gm.n_nodes))
    for r, p in enumerate(plans):
        l2g = p["local_to_global"]
        k = p["n_own"]
        assert np.array_equal(l2g[:k], np.nonzero(part == r)[0])
        assert np.all(np.diff(l2g[k:]) > 0)  # ghosts in global order
        # local cells = cells with an owned node
        has_own = (part[gm.cells] == r).any(axis=1)
        assert np.array_equal(p["cells"], np.nonzero(has_own)[0])
        ghosts = np.setdiff1d(np.unique(gm.cells[has_own]), np.nonzero(part == r)[0])
        assert np.array_equal(l2g[k:], ghosts)
        # lists
        for s in p["neighbors"]:
            s = int(s)
            q = plans[s]
            snd = l2g[p["send"][s]]
            rcv_on_s = q["local_to_global"][q["recv"][r]]
            assert np.array_equal(snd, rcv_on_s)
            assert np.all(p["send"][s] < k)  # owned
            rcv = l2g[p["recv"][s]]
            assert np.all(p["recv"][s] >= k) and np.all(part[rcv] == s)
        # every ghost is received from its owner exactly once
        allr = np.concatenate([p["recv"][int(s)] for s in p["neighbors"]]) if len(p["neighbors"]) else np.zeros(0)
        assert np.array_equal(np.sort(allr), np.arange(k, l2g.size))


@pytest.mark.parametrize("name", ["sphere_cut.msh", "L-shape.msh"])
def test_distributed_spmv_through_the_plan_equals_global(name):
    gm = _mesh(name)
    nparts = 3
    part = af.partition_rcb(gm.dim, gm.coords, nparts)
    rp, cols = O.sparsity(gm.n_nodes, gm.n_nodes, gm.cells)
    vals, _ = O.assemble_poisson(gm.n_nodes, gm.cells, gm.coords, rp, cols, 0.0)
    x = np.random.default_rng(7).standard_normal(gm.n_nodes)
    y_glob = np.array([vals[rp[i]:rp[i + 1]] @ x[cols[rp[i]:rp[i + 1]]] for i in range(gm.n_nodes)])
    plans = [af.subdomain_plan(gm.cells, part, nparts, r) for r in range(nparts)]
    xs = [x[p["local_to_global"][:p["n_own"]]] for p in plans]  # owned values only
    for r, p in enumerate(plans):
        l2g, k = p["local_to_global"], p["n_own"]
        xl = np.full(l2g.size, np.nan)
        xl[:k] = xs[r]
        for s in p["neighbors"]:  # the halo: values packed by the owner from its send list
            s = int(s)
            xl[p["recv"][s]] = xs[s][plans[s]["send"][r]]
        assert not np.isnan(xl).any()
        lc = gm.cells[p["cells"]]
        g2l = np.full(gm.n_nodes, -1, dtype=np.int64)
        g2l[l2g] = np.arange(l2g.size)
        lcells = g2l[lc].astype(np.int32)
        lrp, lcols = O.sparsity(l2g.size, k, lcells)
        lvals, _ = O.assemble_poisson(k, lcells, gm.coords[l2g], lrp, lcols, 0.0)
        yl = np.array([lvals[lrp[i]:lrp[i + 1]] @ xl[lcols[lrp[i]:lrp[i + 1]]] for i in range(k)])
        assert np.abs(yl - y_glob[l2g[:k]]).max() <= 1e-12 * np.abs(y_glob).max()


def test_plan_rejects_bad_input():
    gm = _mesh("L-shape.msh")
    part = np.zeros(gm.n_nodes, dtype=np.int32)
    part[0] = 5
    with pytest.raises(af.AfemError):
        af.subdomain_plan(gm.cells, part, 2, 0)
    with pytest.raises(af.AfemError):
        af.subdomain_plan(gm.cells, np.zeros(gm.n_nodes, dtype=np.int32), 2, 2)
    with pytest.raises(af.AfemError):
        af.partition_rcb(gm.dim, gm.coords, 0)
