"""The Arcane-side shim (shim/AfemDoFLinearSystem.cc, shim/BSRFormat.h) driven the
way an ArcaneFEM module drives its linear-system service, on the GPU, against
the single-subdomain Arcane mock (tests/arcane_mock/: test infrastructure, not
Arcane; tests/arcane_mock/shim_driver.cpp says what each flow does):

  csr  -- setCSRValues with a host CSR + the module's penalty BC variables +
          solve() (HypreDoFLinearSystemImpl semantics, femutils/HypreDoFLinearSystem.cc:138-156, 319-382);
  add  -- matrixAddValue per entry + eliminateRow (AlephDoFLinearSystemImpl, :192-246);
  bsr  -- the shim's BSRFormat<1>: initialize / computeSparsity /
          assembleBilinear(device element lambda) / toLinearSystem (device CSR
          view) / penalty / solve() (modules/poisson/FemModule.cc:261-272).

Case: the reference's sphere_3D Poisson regression (golden_cases.CASES), with
the oracle's system as the expected one; every flow must also meet the
reference golden at checkNodeResultFile's 1e-4 (modules/poisson/FemModule.cc:404).
"""
import os
import subprocess

import numpy as np
import pytest

from arcanefem_amd.gmsh import read_gmsh, read_node_result_file
from golden_cases import CASES, path
from oracle import oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "arcane_mock", "shim_driver")


def _write_case(fname, gm, f, dirichlet, value, coef=1.0):
    n = gm.n_nodes
    rp, cols = O.sparsity(n, n, gm.cells)
    vals, rhs = O.assemble_poisson(n, gm.cells, gm.coords, rp, cols, f)
    with open(fname, "wb") as fh:
        fh.write(np.array([3, 4], np.int32).tobytes())
        fh.write(np.array([n, gm.cells.shape[0]], np.int64).tobytes())
        fh.write(np.ascontiguousarray(gm.coords, np.float64).tobytes())
        fh.write(np.ascontiguousarray(gm.cells, np.int32).tobytes())
        fh.write(np.array([dirichlet.size], np.int64).tobytes())
        fh.write(np.ascontiguousarray(dirichlet, np.int32).tobytes())
        fh.write(np.array([value], np.float64).tobytes())
        fh.write(np.array([cols.size], np.int64).tobytes())
        fh.write(rp.astype(np.int32).tobytes())
        fh.write(cols.astype(np.int32).tobytes())
        fh.write(vals.astype(np.float64).tobytes())
        fh.write(rhs.astype(np.float64).tobytes())
        fh.write(np.array([coef], np.float64).tobytes())
    return rp, cols, vals, rhs


def test_shim_flows_match_oracle_and_golden(tmp_path):
    assert os.path.exists(EXE), "tests/arcane_mock/shim_driver not built (__graft_entry__.build())"
    mfile, f, bcs, gfile, P = CASES["sphere_3D"]
    gm = read_gmsh(path(mfile))
    (group, value), = bcs
    dirichlet = gm.group_nodes(group).astype(np.int32)
    case, out = tmp_path / "case.bin", tmp_path / "out.bin"
    rp, cols, vals, rhs = _write_case(str(case), gm, f, dirichlet, value)
    r = subprocess.run([EXE, str(case), str(out)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, AFEM_OPT_RTOL="1e-14", AFEM_OPT_SOLVER="pcg", AFEM_OPT_MAX_ITER="20000"))
    assert r.returncode == 0, r.stderr
    n = gm.n_nodes
    x = np.fromfile(str(out), np.float64)
    assert x.size == 3 * n
    x_csr, x_add, x_bsr = x[:n], x[n:2 * n], x[2 * n:]
    # expected: the oracle's systems, solved directly
    pv, pr = vals.copy(), rhs.copy()
    O.dirichlet_penalty(dirichlet, value, P, rp, cols, pv, pr)
    xp = np.linalg.solve(O.csr_to_dense(rp, cols, pv), pr)
    ev, er = vals.copy(), rhs.copy()
    O.row_elimination(dirichlet, value, rp, cols, ev, er)
    xe = np.linalg.solve(O.csr_to_dense(rp, cols, ev), er)
    scale = np.abs(xp).max()
    assert np.abs(x_csr - xp).max() / scale <= 1e-10
    assert np.abs(x_bsr - xp).max() / scale <= 1e-10
    assert np.abs(x_add - xe).max() / scale <= 1e-10
    gold = read_node_result_file(path(gfile))
    for x_ in (x_csr, x_add, x_bsr):
        nerr, _ = O.check_node_result({int(t): x_[i] for i, t in enumerate(gm.node_tags)}, gold, 1e-4)
        assert nerr == 0


E3, NU3 = 21.0e5, 0.28
LAM3, MU3 = E3 * NU3 / ((1 + NU3) * (1 - 2 * NU3)), E3 / (2 * (1 + NU3))
BODY3 = np.array([0.5, -0.25, -1.0])


def _write_rank_case(fname, n, cells, coords, own, nbr, shared, ghosts, dirichlet, value, rows, cols, vals, rhs,
                     rhs3):
    with open(fname, "wb") as fh:
        fh.write(np.array([n, cells.shape[0]], np.int64).tobytes())
        fh.write(np.ascontiguousarray(coords, np.float64).tobytes())
        fh.write(np.ascontiguousarray(cells, np.int32).tobytes())
        fh.write(np.ascontiguousarray(own, np.uint8).tobytes())
        fh.write(np.array([len(nbr)], np.int32).tobytes())
        for r in nbr:
            fh.write(np.array([r], np.int32).tobytes())
            fh.write(np.array([shared[r].size], np.int64).tobytes())
            fh.write(np.ascontiguousarray(shared[r], np.int32).tobytes())
            fh.write(np.array([ghosts[r].size], np.int64).tobytes())
            fh.write(np.ascontiguousarray(ghosts[r], np.int32).tobytes())
        fh.write(np.array([dirichlet.size], np.int64).tobytes())
        fh.write(np.ascontiguousarray(dirichlet, np.int32).tobytes())
        fh.write(np.array([value], np.float64).tobytes())
        fh.write(np.array([cols.size], np.int64).tobytes())
        fh.write(np.ascontiguousarray(rows, np.int32).tobytes())
        fh.write(np.ascontiguousarray(cols, np.int32).tobytes())
        fh.write(np.ascontiguousarray(vals, np.float64).tobytes())
        fh.write(np.ascontiguousarray(rhs, np.float64).tobytes())
        fh.write(np.ascontiguousarray(rhs3, np.float64).tobytes())
        fh.write(np.array([LAM3, MU3], np.float64).tobytes())


def _dense_blocks(rp, cols, vals, k):
    """Per-block k x k values -> the dense scalar matrix."""
    n = rp.shape[0] - 1
    A = np.zeros((k * n, k * n))
    for r in range(n):
        for t in range(rp[r], rp[r + 1]):
            A[k * r:k * r + k, k * cols[t]:k * cols[t] + k] = vals[k * k * t:k * k * (t + 1)].reshape(k, k)
    return A


@pytest.mark.parametrize("world", [1, 2, 3])
def test_shim_subdomains_over_the_parallel_mng(tmp_path, world):
    """The shim on `world` subdomains (threads sharing the mock's MockWorld,
    transport = "host": libafem's halo and reductions go through the shim's
    IParallelMng transport).  Each subdomain has Arcane-style local ids --
    owned and ghost DoFs interleaved by a random permutation -- so the shim's
    numbering (_computeNumbering), its permuted setCSRValues copy, the halo
    built from the DoF family's IVariableSynchronizer lists (_buildHalo,
    FemDoFsOnNodes.cc:125-126) and the solution's synchronize() all run.  The
    partition is libafem's RCB with its subdomain plan (the lists Arcane's
    ghost layer would give).  The same again through the shim's BSRFormat<1>
    and BSRFormat<3> (block-3 elasticity, body force, clamped nodes)
    (initialize / computeSparsity / assembleBilinear(element lambda) on the
    cell-unit kernel / toLinearSystem: a device CSR view in the subdomain's
    DoF numbering, renumbered on the device by the linear system) on each
    subdomain.  Owned values equal the single-domain oracle solve to 1e-10,
    every ghost its owner's value bit for bit."""
    import arcanefem_amd as af

    assert os.path.exists(EXE), "tests/arcane_mock/shim_driver not built (__graft_entry__.build())"
    mfile, f, bcs, gfile, P = CASES["sphere_3D"]
    gm = read_gmsh(path(mfile))
    (group, value), = bcs
    is_dir = np.zeros(gm.n_nodes, bool)
    is_dir[gm.group_nodes(group)] = True
    part = af.partition_rcb(3, gm.coords, world)
    rng = np.random.default_rng(7 + world)
    l2g_arc = []
    for r in range(world):
        plan = af.subdomain_plan(gm.cells, part, world, r)
        l2g, n_own = plan["local_to_global"], plan["n_own"]
        n = l2g.size
        g2l = np.full(gm.n_nodes, -1, np.int64)
        g2l[l2g] = np.arange(n)
        lcells = g2l[gm.cells[plan["cells"]]].astype(np.int32)
        rp, cols = O.sparsity(n, n_own, lcells)  # libafem-local numbering: owned rows first
        vals, rhs = O.assemble_poisson(n_own, lcells, gm.coords[l2g], rp, cols, f)
        pi = rng.permutation(n)  # libafem-local index -> Arcane local id
        inv = np.argsort(pi)
        rows_a, cols_a, vals_a = [0], [], []
        for L in range(n):
            a = inv[L]
            if a < n_own:
                c = pi[cols[rp[a]:rp[a + 1]]]
                o = np.argsort(c)
                cols_a.extend(c[o])
                vals_a.extend(vals[rp[a]:rp[a + 1]][o])
            rows_a.append(len(cols_a))
        own = inv < n_own
        rhs_a = np.where(own, rhs[np.minimum(inv, n_own - 1)], 0.0)
        _, rhs3 = O.assemble_elasticity_tet(n_own, lcells, gm.coords[l2g], rp, cols, LAM3, 2 * MU3, 0.0, BODY3)
        rhs3_a = np.where(own[:, None], rhs3.reshape(-1, 3)[np.minimum(inv, n_own - 1)], 0.0).ravel()
        dirichlet = np.flatnonzero(own & is_dir[l2g[inv]]).astype(np.int32)
        nbr = [int(x) for x in plan["neighbors"]]
        _write_rank_case(str(tmp_path / f"case{r}.bin"), n, pi[lcells].astype(np.int32), gm.coords[l2g[inv]], own,
                         nbr, {q: pi[plan["send"][q]] for q in nbr}, {q: pi[plan["recv"][q]] for q in nbr},
                         dirichlet, value, np.array(rows_a), np.array(cols_a), np.array(vals_a), rhs_a, rhs3_a)
        l2g_arc.append((l2g[inv], own))
    r = subprocess.run([EXE, "par", str(world), str(tmp_path / "case"), str(tmp_path / "out")], capture_output=True,
                       text=True, timeout=180,
                       env=dict(os.environ, AFEM_OPT_RTOL="1e-14", AFEM_OPT_SOLVER="pcg", AFEM_OPT_MAX_ITER="20000",
                                AFEM_OPT_TRANSPORT="host", AFEM_MOCK_TRACE="1"))
    print(r.stderr[-3000:])  # the shim's info() trace (shown when the test fails)
    assert r.returncode == 0, r.stderr
    # the single-domain system, solved directly
    n = gm.n_nodes
    rp, cols = O.sparsity(n, n, gm.cells)
    vals, rhs = O.assemble_poisson(n, gm.cells, gm.coords, rp, cols, f)
    O.dirichlet_penalty(np.flatnonzero(is_dir).astype(np.int32), value, P, rp, cols, vals, rhs)
    xg = np.linalg.solve(O.csr_to_dense(rp, cols, vals), rhs)
    # BSRFormat<3>: the block-3 elasticity system, clamped on the Dirichlet nodes by penalty
    ev, erhs = O.assemble_elasticity_tet(n, gm.cells, gm.coords, rp, cols, LAM3, 2 * MU3, 0.0, BODY3)
    A3 = _dense_blocks(rp, cols, ev, 3)
    clamp = (3 * np.flatnonzero(is_dir)[:, None] + np.arange(3)).ravel()
    A3[clamp, clamp] = 1.0e30
    erhs[clamp] = 0.0
    x3 = np.linalg.solve(A3, erhs).reshape(-1, 3)
    # the setCSRValues flow, the shim's BSRFormat<1>, then its BSRFormat<3> on the same subdomains
    for flow, k, xref in ((0, 1, xg[:, None]), (1, 1, xg[:, None]), (2, 3, x3)):
        owner_val = np.full((n, k), np.nan)
        xs = []
        for q in range(world):
            xq = np.fromfile(str(tmp_path / f"out{q}.bin"), np.float64)
            g, own = l2g_arc[q]
            assert xq.size == 5 * g.size
            x = xq[flow * g.size:flow * g.size + k * g.size].reshape(-1, k)
            owner_val[g[own]] = x[own]
            xs.append((x, g, own))
        assert not np.isnan(owner_val).any()
        assert np.abs(owner_val - xref).max() <= 1e-10 * np.abs(xref).max(), flow
        for x, g, own in xs:
            assert np.array_equal(x[~own], owner_val[g[~own]])  # synchronize(): ghosts hold their owners' values
