"""GPU tests through the C ABI of the boundary terms, the direct solver, the
fallback assembly kernels and the plugin entry points not exercised by
test_gpu_parity.py.

Reference semantics (toutane/arcanefem @ 2025-02-20):
  * Neumann / traction RHS: femutils/ArcaneFemFunctionsGpu.h:612-766,
    modules/elasticity/FemModule.cc:244-273; pinned by the reference goldens
    poisson_test_ref_{circle,sphere}_neumann_*.txt and
    elasticity_traction_bar_test_ref.txt (oracle replay: test_oracle_golden.py);
  * constant source accumulates (doAtomic<Add>, ArcaneFemFunctionsGpu.h:419-428);
  * direct branch of the Sequential solver below 500 rows (DoFLinearSystem.cc:127-136);
  * eliminateRow / eliminateRowColumn: Aleph _fillMatrix (AlephDoFLinearSystem.cc:501-583);
  * BSRMatrix::toCsr layout (BSRFormat.h:194-256), getValue / setValue /
    resetMatrixValues, clearValues (HypreDoFLinearSystem.cc:180-187).
Tolerances: matrix / RHS entries 1e-12 x max|oracle|; solutions 1e-10
relative (max norm) against the oracle's dense solve; goldens at the
restatement's measured error (x ~1e3 headroom) and the reference's own gate.
"""
import numpy as np
import pytest

import arcanefem_amd as af
from arcanefem_amd.gmsh import read_gmsh, read_node_result_file
from oracle import oracle as O

from golden_cases import CASES, ELASTICITY_BAR, NEUMANN_CASES, lame, path

pytestmark = pytest.mark.gpu

VAL_TOL = 1e-12
SOL_TOL = 1e-10
K_STRIP, K_TILE, K_GLOBAL, K_E3_STRIP, K_E3_ITEM, K_E3_GLOBAL, K_E2, K_E3_WG, K_E3_BIG = 1, 2, 3, 4, 5, 6, 7, 8, 9


def _close(a, b, tol=VAL_TOL):
    scale = max(np.abs(b).max(), 1e-300)
    err = np.abs(a - b).max() / scale
    assert err <= tol, f"differ from the oracle: {err:.3e}"
    return err


# ---------------------------------------------------------------- Neumann (K15)
@pytest.mark.parametrize("case", list(NEUMANN_CASES))
@pytest.mark.parametrize("method", ["direct", "pcg"])
def test_neumann_golden(ctx, case, method):
    mfile, f, dirichlet, neumann, gfile, P = NEUMANN_CASES[case]
    gm = read_gmsh(path(mfile))
    mesh = af.Mesh.from_arrays(ctx, gm.dim, gm.cells, gm.coords)
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    bsr.computeSparsity()
    ls = af.DoFLinearSystem().initialize(ctx, gm.n_nodes)
    bsr.assemblePoissonP1(1.0, f, ls.rhsVariable())
    bsr.toLinearSystem(ls)
    orp, ocols = O.sparsity(gm.n_nodes, gm.n_nodes, gm.cells)
    ovals, orhs = O.assemble_poisson(gm.n_nodes, gm.cells, gm.coords, orp, ocols, f)
    for g, v in neumann:
        faces = gm.group_faces(g)
        fc = gm.face_cells(faces)
        af.applyNeumannToRhs(mesh, ls.rhsVariable(), faces, v, "normal", 1, fc)
        O.neumann(gm.dim, gm.n_nodes, 1, O.NEUMANN_NORMAL, v, faces, fc, gm.cells, gm.coords, orhs)
    _close(ls.rhs_host(), orhs)
    for g, v in dirichlet:
        ls.applyDirichletViaPenalty(gm.group_nodes(g), v, P)
        O.dirichlet_penalty(gm.group_nodes(g), v, P, orp, ocols, ovals, orhs)
    ls.setSolverOptions(method=method, rtol=1e-14, max_iter=20000)
    st = ls.solve()
    assert st["converged"], st
    x = ls.solution_host()
    xo = np.linalg.solve(O.csr_to_dense(orp, ocols, ovals), orhs)
    assert np.abs(x - xo).max() / np.abs(xo).max() <= SOL_TOL
    gold = read_node_result_file(path(gfile))
    nerr, mx = O.check_node_result({int(t): x[i] for i, t in enumerate(gm.node_tags)}, gold, 1e-4)
    print(f"{case} [{method}]: max rel error vs reference golden {mx:.3e} ({st['iterations']} iterations)")
    assert nerr == 0 and mx <= 1e-10


def test_neumann_value_mode_and_ghost_nodes(ctx):
    # scalar flux g * |F| / nf on the faces of the z=0 plane of a slab with
    # ghosts: only owned nodes receive a share (nodes_infos.isOwn)
    mesh = af.Mesh.structured(ctx, 3, 5, nz=7, nranks=2, rank=1)
    cells, coords, _ = mesh.download()
    # boundary faces of the slab's top: tets faces with all nodes at z = 7/5 (the box top)
    zmax = coords[:, 2].max()
    top = np.abs(coords[:, 2] - zmax) < 0.3 / 5
    faces = []
    for c in cells:
        for a in range(4):
            f = np.delete(c, a)
            if top[f].all():
                faces.append(f)
    faces = np.unique(np.sort(np.array(faces, dtype=np.int32), axis=1), axis=0)
    assert faces.shape[0] == 2 * 5 * 5
    n_own = mesh.n_own_nodes
    drhs = ctx.malloc(8 * n_own)
    ctx.to_device(drhs, np.zeros(n_own))
    af.applyNeumannToRhs(mesh, drhs, faces, 2.5, "value")
    rhs = ctx.to_host(drhs, n_own, np.float64)
    ctx.free(drhs)
    orhs = O.neumann(3, n_own, 1, O.NEUMANN_VALUE, 2.5, faces, None, cells, coords, np.zeros(n_own))
    _close(rhs, orhs)
    assert abs(rhs.sum() - 2.5 * 1.0) < 0.05  # the flux times the (jittered) top area


@pytest.mark.parametrize("use_csr", [False, True])
@pytest.mark.parametrize("method", ["direct", "pcg"])
def test_elasticity_traction_bar_golden(ctx, use_csr, method):
    """Block-2 elasticity with traction, pinned by the reference's elasticity golden."""
    c = ELASTICITY_BAR
    gm = read_gmsh(path(c["mesh"]))
    lam, mu2 = lame(c["E"], c["nu"])
    n = gm.n_nodes
    mesh = af.Mesh.from_arrays(ctx, 2, gm.cells, gm.coords)
    bsr = af.BSRFormat(mesh, 2).initialize(use_csr)
    bsr.computeSparsity()
    bsr.assembleElasticityP1(lam, mu2)
    assert bsr.stats()["last_kernel"] == K_E2
    ls = af.DoFLinearSystem().initialize(ctx, 2 * n)
    bsr.toLinearSystem(ls)
    faces = gm.group_faces(c["traction_group"])
    af.applyNeumannToRhs(mesh, ls.rhsVariable(), faces, c["traction"], "traction", nb_dof=2)
    orhs = O.neumann(2, n, 2, O.NEUMANN_TRACTION, c["traction"], faces, None, gm.cells, gm.coords, np.zeros(2 * n))
    _close(ls.rhs_host(), orhs)
    clamp = gm.group_nodes(c["clamp"])
    dofs = np.concatenate([2 * clamp, 2 * clamp + 1]).astype(np.int32)
    ls.applyDirichletViaPenalty(dofs, 0.0, c["penalty"])
    ls.setSolverOptions(method=method, rtol=1e-15, max_iter=50000)
    st = ls.solve()
    u = ls.solution_host()
    gold = read_node_result_file(path(c["golden"]))
    worst, nerr = 0.0, 0
    for comp in range(2):
        g = {uid: val[comp] for uid, val in gold.items()}
        e, mx = O.check_node_result({int(t): u[2 * i + comp] for i, t in enumerate(gm.node_tags)}, g, 1e-3, 1e-16)
        nerr += e
        worst = max(worst, mx)
    print(f"bar traction [{method}, csr={use_csr}]: max rel error vs golden {worst:.3e}, {st}")
    assert nerr == 0
    assert worst <= (1e-10 if method == "direct" else 1e-6)


# ---------------------------------------------------------------- RHS semantics
def test_rhs_source_accumulates_like_the_reference(ctx):
    mesh = af.Mesh.structured(ctx, 3, 6)
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    bsr.computeSparsity()
    ls = af.DoFLinearSystem().initialize(ctx, mesh.n_own_nodes)
    bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable())
    r1 = ls.rhs_host()
    bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable())
    assert np.array_equal(ls.rhs_host(), 2.0 * r1)
    bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable(), rhs_mode="set")
    assert np.array_equal(ls.rhs_host(), r1)
    mesh3 = af.Mesh.structured(ctx, 3, 4)
    b3 = af.BSRFormat(mesh3, 3).initialize(False)
    b3.computeSparsity()
    n3 = 3 * mesh3.n_own_nodes
    d = ctx.malloc(8 * n3)
    ctx.to_device(d, np.ones(n3))
    b3.assembleElasticityP1Ex(1.0, 2.0, 0.0, (1.0, 2.0, 3.0), d)
    ra = ctx.to_host(d, n3, np.float64)
    b3.assembleElasticityP1Ex(1.0, 2.0, 0.0, (1.0, 2.0, 3.0), d, rhs_mode="set")
    rs = ctx.to_host(d, n3, np.float64)
    ctx.free(d)
    assert np.array_equal(ra, 1.0 + rs)


# ---------------------------------------------------------------- solvers
@pytest.mark.parametrize("case", ["circle_2D", "sphere_3D", "L-shape_3D"])
def test_direct_and_pcg_agree(ctx, case):
    mfile, f, bcs, gfile, P = CASES[case]
    gm = read_gmsh(path(mfile))
    sols = {}
    for method in ("auto", "direct", "pcg"):
        mesh = af.Mesh.from_arrays(ctx, gm.dim, gm.cells, gm.coords)
        bsr = af.BSRFormat(mesh, 1).initialize(True)
        bsr.computeSparsity()
        ls = af.DoFLinearSystem().initialize(ctx, gm.n_nodes)
        bsr.assemblePoissonP1(1.0, f, ls.rhsVariable())
        bsr.toLinearSystem(ls)
        for g, v in bcs:
            ls.applyDirichletViaPenalty(gm.group_nodes(g), v, P)
        ls.setSolverOptions(method=method, rtol=1e-14, max_iter=20000)
        st = ls.solve()
        assert st["converged"]
        if method != "pcg":
            assert st["iterations"] == 0  # n < 500: the Sequential solver's direct branch
        sols[method] = ls.solution_host()
    assert np.array_equal(sols["auto"], sols["direct"])
    assert np.abs(sols["direct"] - sols["pcg"]).max() <= SOL_TOL * np.abs(sols["direct"]).max()


def test_direct_solver_limit_and_singular(ctx):
    ls = af.DoFLinearSystem().initialize(ctx, 3)
    ls.matrixAddValue(0, 0, 1.0)
    ls.matrixAddValue(1, 1, 2.0)  # row 2 empty: singular
    ls.set_rhs_host(np.ones(3))
    ls.setSolverOptions(method="direct")
    with pytest.raises(af.AfemError):
        ls.solve()


# ---------------------------------------------------------------- elimination (Aleph semantics)
@pytest.mark.parametrize("method", ["direct", "pcg"])
def test_eliminate_row_and_row_column(ctx, method):
    gm = read_gmsh(path("circle_cut.msh"))
    n = gm.n_nodes
    mesh = af.Mesh.from_arrays(ctx, 2, gm.cells, gm.coords)
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    bsr.computeSparsity()
    ls = af.DoFLinearSystem().initialize(ctx, n)
    bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable())
    bsr.toLinearSystem(ls)
    rc = gm.group_nodes("horizontal")
    row_only = np.setdiff1d(gm.group_nodes("curved"), rc)[::3]
    for d in rc:
        ls.eliminateRowColumn(int(d), 0.5)
    for d in row_only:
        ls.eliminateRow(int(d), -0.25)
    ls.setSolverOptions(method=method, rtol=1e-14, max_iter=20000)
    st = ls.solve()
    assert st["converged"]
    x = ls.solution_host()
    orp, ocols = O.sparsity(n, n, gm.cells)
    ovals, orhs = O.assemble_poisson(n, gm.cells, gm.coords, orp, ocols, 5.5)
    info = np.zeros(n, np.uint8)
    val = np.zeros(n)
    info[rc], val[rc] = 2, 0.5
    info[row_only], val[row_only] = 1, -0.25
    O.eliminate(info, val, orp, ocols, ovals, orhs)
    _, _, vals = bsr.download()
    _close(vals, ovals)  # the matrix after _fillMatrix's elimination
    xo = np.linalg.solve(O.csr_to_dense(orp, ocols, ovals), orhs)
    assert np.abs(x - xo).max() / np.abs(xo).max() <= SOL_TOL
    assert np.all(x[rc] == 0.5) and np.all(x[row_only] == -0.25)


# ---------------------------------------------------------------- plugin entry points
def _mesh_for_k(ctx, k):
    if k == 2:
        return af.Mesh.structured(ctx, 2, 7)
    return af.Mesh.structured(ctx, 3, 4 if k == 3 else 5)


def _assemble_k(bsr, k):
    if k == 1:
        bsr.assemblePoissonP1(1.0, 0.0, None)
    elif k == 2:
        bsr.assembleElasticityP1(1.2e5, 1.6e5)
    else:
        bsr.assembleElasticityP1Ex(1.2e5, 1.6e5, 0.0, None, None)


def _oracle_blocks(mesh, k):
    cells, coords, _ = mesh.download()
    orp, ocols = O.sparsity(mesh.n_nodes, mesh.n_own_nodes, cells)
    if k == 1:
        ov, _ = O.assemble_poisson(mesh.n_own_nodes, cells, coords, orp, ocols, 0.0)
    elif k == 2:
        ov = O.assemble_elasticity_tri(mesh.n_own_nodes, cells, coords, orp, ocols, 1.2e5, 1.6e5)
    else:
        ov, _ = O.assemble_elasticity_tet(mesh.n_own_nodes, cells, coords, orp, ocols, 1.2e5, 1.6e5, 0.0, None)
    return orp, ocols, ov


@pytest.mark.parametrize("k", [1, 2, 3])
@pytest.mark.parametrize("use_csr", [False, True])
def test_export_csr32_matches_tocsr_layout(ctx, k, use_csr):
    """BSRMatrix::toCsr (femutils/BSRFormat.h:194-256): scalar row s = br*k + i
    starts at rows_b[br]*k^2 + i*k*len, its columns are cols_b*k + j in block
    order, values in that order; rows without the n+1 sentinel."""
    mesh = _mesh_for_k(ctx, k)
    bsr = af.BSRFormat(mesh, k).initialize(use_csr)
    bsr.computeSparsity()
    _assemble_k(bsr, k)
    rows, rnc, cols, vals = bsr.export_csr32()
    orp, ocols, ov = _oracle_blocks(mesh, k)
    nb = orp.shape[0] - 1
    erows, ernc, ecols, evals = [], [], [], []
    for br in range(nb):
        b0, b1 = orp[br], orp[br + 1]
        blk = ov[k * k * b0:k * k * b1].reshape(b1 - b0, k, k)
        for i in range(k):
            erows.append(k * k * b0 + i * k * (b1 - b0))
            ernc.append(k * (b1 - b0))
            for t in range(b1 - b0):
                for j in range(k):
                    ecols.append(ocols[b0 + t] * k + j)
                    evals.append(blk[t, i, j])
    assert np.array_equal(rows, np.array(erows)) and np.array_equal(rnc, np.array(ernc))
    assert np.array_equal(cols, np.array(ecols))
    _close(vals, np.array(evals))


@pytest.mark.parametrize("k", [1, 2, 3])
def test_get_set_reset_values(ctx, k):
    mesh = _mesh_for_k(ctx, k)
    bsr = af.BSRFormat(mesh, k).initialize(k != 2)
    bsr.computeSparsity()
    _assemble_k(bsr, k)
    rows, rnc, cols, vals = bsr.export_csr32()
    rng = np.random.default_rng(5)
    for s in rng.integers(0, rows.shape[0], 12):
        t = rows[s] + rng.integers(0, rnc[s])
        assert bsr.getValue(int(s), int(cols[t])) == vals[t]
        bsr.setValue(int(s), int(cols[t]), 7.25)
        assert bsr.getValue(int(s), int(cols[t])) == 7.25
    bsr.resetMatrixValues()
    _, _, v2 = bsr.download()
    assert not v2.any()
    with pytest.raises(af.AfemError) as e:
        bsr.getValue(0, k * (mesh.n_nodes - 1))  # far corner: not in the structure
    assert e.value.code == 5


def test_clear_values_then_reassemble(ctx):
    gm = read_gmsh(path("L-shape.msh"))
    n = gm.n_nodes
    mesh = af.Mesh.from_arrays(ctx, 2, gm.cells, gm.coords)
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    bsr.computeSparsity()
    ls = af.DoFLinearSystem().initialize(ctx, n)
    ls.applyDirichletViaPenalty(gm.group_nodes("boundary"), 0.5, 1e30)
    ls.eliminateRow(0, 1.0)
    ls.clearValues()  # drops the view, the forced / elimination flags
    with pytest.raises(af.AfemError) as e:
        ls.solve()
    assert e.value.code == 4
    assert not ctx.to_host(ls.getForcedInfo(), n, np.uint8).any()
    assert not ctx.to_host(ls.getEliminationInfo(), n, np.uint8).any()
    bsr.assemblePoissonP1(1.0, -5.5, ls.rhsVariable(), rhs_mode="set")
    bsr.toLinearSystem(ls)
    ls.applyDirichletViaPenalty(gm.group_nodes("boundary"), 0.5, 1e30)
    st = ls.solve()
    x = ls.solution_host()
    gold = read_node_result_file(path("poisson_test_ref_L-shape_2D.txt"))
    nerr, mx = O.check_node_result({int(t): x[i] for i, t in enumerate(gm.node_tags)}, gold, 1e-4)
    assert st["converged"] and nerr == 0 and mx < 1e-10


def test_host_csr_view_accepts_point_updates(ctx):
    """setCSRValues from host memory, then matrixAddValue / matrixSetValue on
    entries of the view (HypreDoFLinearSystem.cc:148-156): the updates land in
    the view and the solve sees the full matrix (capi.cpp:650)."""
    gm = read_gmsh(path("circle_cut.msh"))
    n = gm.n_nodes
    orp, ocols = O.sparsity(n, n, gm.cells)
    ovals, orhs = O.assemble_poisson(n, gm.cells, gm.coords, orp, ocols, 5.5)
    ls = af.DoFLinearSystem().initialize(ctx, n)
    ls.setCSRValues(orp[:-1].astype(np.int32), np.diff(orp).astype(np.int32), ocols, ovals)
    ls.set_rhs_host(orhs)
    r = 7
    t = orp[r] + 1
    ls.matrixAddValue(r, int(ocols[t]), 0.125)
    ovals[t] += 0.125
    for d in gm.group_nodes("horizontal"):
        ls.matrixSetValue(int(d), int(d), 1e30)
    ls.set_rhs_host(np.where(np.isin(np.arange(n), gm.group_nodes("horizontal")), 0.5e30, orhs))
    O.dirichlet_penalty(gm.group_nodes("horizontal"), 0.5, 1e30, orp, ocols, ovals, orhs)
    with pytest.raises(af.AfemError):
        ls.matrixAddValue(0, n - 1, 1.0)  # outside the view's structure
    ls.setSolverOptions(method="direct")
    st = ls.solve()
    x = ls.solution_host()
    xo = np.linalg.solve(O.csr_to_dense(orp, ocols, ovals), orhs)
    assert st["converged"] and np.abs(x - xo).max() / np.abs(xo).max() <= SOL_TOL


def test_host_csr_view_is_read_at_solve(ctx):
    """The view contract of femutils/DoFLinearSystem.h:251-258: a host CSR view
    stays the matrix until solve.  The module edits its own value array after
    setCSRValues (no matrixAddValue call); the solve must see the edit, as
    Hypre's solve reads the live view (HypreDoFLinearSystem.cc:587-599)."""
    gm = read_gmsh(path("circle_cut.msh"))
    n = gm.n_nodes
    orp, ocols = O.sparsity(n, n, gm.cells)
    ovals, orhs = O.assemble_poisson(n, gm.cells, gm.coords, orp, ocols, 5.5)
    O.dirichlet_penalty(gm.group_nodes("horizontal"), 0.5, 1e30, orp, ocols, ovals, orhs)
    vals = ovals.copy()
    ls = af.DoFLinearSystem().initialize(ctx, n)
    ls.setCSRValues(orp[:-1].astype(np.int32), np.diff(orp).astype(np.int32), ocols, vals)
    ls.set_rhs_host(orhs)
    # the module's own edit after the hand-over: a mass-like shift of every diagonal
    diag = np.array([orp[r] + np.searchsorted(ocols[orp[r]:orp[r + 1]], r) for r in range(n)])
    free = vals[diag] < 1e20
    vals[diag[free]] += 3.0
    ovals[diag[free]] += 3.0
    ls.setSolverOptions(method="direct")
    st = ls.solve()
    x = ls.solution_host()
    xo = np.linalg.solve(O.csr_to_dense(orp, ocols, ovals), orhs)
    assert st["converged"] and np.abs(x - xo).max() / np.abs(xo).max() <= SOL_TOL


@pytest.mark.parametrize("method", ["direct", "pcg"])
def test_host_csr_view_apply_bcs_then_solve(ctx, method):
    """ADVICE r3 (capi.cpp:1124): on a host CSR view, applyBoundaryConditions
    and then solve() with row+column elimination.  The elimination is applied
    once: it lands in the module's view (as Hypre edits the view's values,
    HypreDoFLinearSystem.cc:319-382) and the solve's second pass is a no-op, so
    b_j -= A_ji g is not subtracted twice."""
    gm = read_gmsh(path("circle_cut.msh"))
    n = gm.n_nodes
    orp, ocols = O.sparsity(n, n, gm.cells)
    ovals, orhs = O.assemble_poisson(n, gm.cells, gm.coords, orp, ocols, 5.5)
    vals = ovals.copy()
    ls = af.DoFLinearSystem().initialize(ctx, n)
    ls.setCSRValues(orp[:-1].astype(np.int32), np.diff(orp).astype(np.int32), ocols, vals)
    ls.set_rhs_host(orhs)
    rc = gm.group_nodes("horizontal")
    for d in rc:
        ls.eliminateRowColumn(int(d), 0.5)
    ls.applyBoundaryConditions()
    info = np.zeros(n, np.uint8)
    val = np.zeros(n)
    info[rc], val[rc] = 2, 0.5
    O.eliminate(info, val, orp, ocols, ovals, orhs)
    _close(vals, ovals)  # the eliminated matrix is in the module's view
    _close(ls.rhs_host(), orhs)
    ls.setSolverOptions(method=method, rtol=1e-14, max_iter=20000)
    st = ls.solve()
    _close(ls.rhs_host(), orhs)  # not corrected a second time
    x = ls.solution_host()
    xo = np.linalg.solve(O.csr_to_dense(orp, ocols, ovals), orhs)
    assert st["converged"] and np.abs(x - xo).max() / np.abs(xo).max() <= SOL_TOL
    assert np.all(x[rc] == 0.5)


def test_duplicate_diagonal_entries_add_up(ctx):
    """ADVICE r4 (linear_system.hip k_inv_diag): a view whose rows repeat the
    (i, i) entry (a module that adds its diagonal in two pieces).  The operator
    applies both (SpMV, csr_to_dense), the Jacobi preconditioner and the
    constraint test use their sum, in libafem and in the oracle alike: a fixed
    number of PCG iterations gives the same iterate on both."""
    gm = read_gmsh(path("circle_cut.msh"))
    n = gm.n_nodes
    orp, ocols = O.sparsity(n, n, gm.cells)
    ovals, orhs = O.assemble_poisson(n, gm.cells, gm.coords, orp, ocols, 5.5)
    O.dirichlet_penalty(gm.group_nodes("horizontal"), 0.5, 1e30, orp, ocols, ovals, orhs)
    # every third row: the diagonal split into 0.25 d (in place) + 0.75 d (appended)
    split = np.arange(0, n, 3)
    rows, cols, vals = [], [], []
    for r in range(n):
        c = list(ocols[orp[r]:orp[r + 1]])
        v = list(ovals[orp[r]:orp[r + 1]])
        if r in set(split.tolist()):
            k = c.index(r)
            d = v[k]
            v[k] = 0.25 * d
            c.append(r)
            v.append(0.75 * d)
        rows.append(len(cols))
        cols += c
        vals += v
    rp = np.array(rows + [len(cols)], dtype=np.int64)
    cols = np.array(cols, dtype=np.int32)
    vals = np.array(vals)
    assert np.allclose(O.csr_to_dense(rp, cols, vals), O.csr_to_dense(orp, ocols, ovals), rtol=1e-15, atol=0)
    ls = af.DoFLinearSystem().initialize(ctx, n)
    ls.setCSRValues(rp[:-1].astype(np.int32), np.diff(rp).astype(np.int32), cols, vals)
    ls.set_rhs_host(orhs)
    ls.setSolverOptions(fixed_iterations=25)
    ls.solve()
    xo, _, _, _ = O.pcg_jacobi(rp, cols, vals, orhs, max_iter=-25)
    xs, _, _, _ = O.pcg_jacobi(orp, ocols, ovals, orhs, max_iter=-25)  # the unsplit system: same iterate
    x = ls.solution_host()
    assert np.abs(xo - xs).max() <= 1e-10 * np.abs(xs).max()
    assert np.abs(x - xo).max() <= 1e-10 * np.abs(xo).max()


def test_mapped_view_rejects_duplicate_and_missing_rows(ctx):
    """ADVICE r4 (handover.hip k_lsmap_len): afem_ls_set_csr_values_mapped with
    a device view in the caller's numbering.  A valid permuted index solves like
    the oracle; an index mapping two caller rows to one linear-system row, or
    leaving an owned row without a caller row, is refused (it used to write one
    row's entries past its range, or leave an empty row)."""
    from arcanefem_amd._capi import call

    gm = read_gmsh(path("circle_cut.msh"))
    n = gm.n_nodes
    orp, ocols = O.sparsity(n, n, gm.cells)
    ovals, orhs = O.assemble_poisson(n, gm.cells, gm.coords, orp, ocols, 5.5)
    O.dirichlet_penalty(gm.group_nodes("horizontal"), 0.5, 1e30, orp, ocols, ovals, orhs)
    rows = orp[:-1].astype(np.int32)
    cols = ocols.astype(np.int32)
    bufs = []

    def dev(a):
        p = ctx.malloc(max(a.nbytes, 8))
        ctx.to_device(p, a)
        bufs.append(p)
        return p

    drows, dcols, dvals = dev(rows), dev(cols), dev(ovals.copy())

    def mapped(index):
        ls = af.DoFLinearSystem().initialize(ctx, n)
        idx = np.ascontiguousarray(index, dtype=np.int32)
        call("afem_ls_set_csr_values_mapped", ls.impl, drows, None, dcols, dvals, n, cols.size,
             idx.ctypes.data, idx.size)
        return ls

    perm = np.random.default_rng(5).permutation(n).astype(np.int32)  # caller dof d -> ls row perm[d]
    ls = mapped(perm)
    b = np.empty(n)
    b[perm] = orhs
    ls.set_rhs_host(b)
    ls.setSolverOptions(method="direct")
    st = ls.solve()
    xo = np.linalg.solve(O.csr_to_dense(orp, ocols, ovals), orhs)
    assert st["converged"] and np.abs(ls.solution_host()[perm] - xo).max() / np.abs(xo).max() <= SOL_TOL
    dup = perm.copy()
    dup[3] = dup[11]  # two caller rows -> one ls row, and ls row perm[3] gets none
    with pytest.raises(af.AfemError, match="two rows"):
        mapped(dup)
    missing = perm.copy()
    missing[7] = -1  # caller row 7 is not owned: its ls row stays empty
    with pytest.raises(af.AfemError, match="no row"):
        mapped(missing)
    for p in bufs:
        ctx.free(p)


def test_boundary_argument_checks(ctx):
    # ADVICE r1 (capi.cpp:544): a subdomain CSR has ghost columns, the linear
    # system must span them
    mesh = af.Mesh.structured(ctx, 3, 4, nz=6, nranks=2, rank=0)
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    bsr.computeSparsity()
    ls = af.DoFLinearSystem().initialize(ctx, mesh.n_own_nodes)
    with pytest.raises(af.AfemError) as e:
        bsr.toLinearSystem(ls)
    assert e.value.code == 1
    ls2 = af.DoFLinearSystem().initialize(ctx, 3)
    with pytest.raises(af.AfemError):
        ls2.setCSRValues(np.array([0, 1, 2]), None, np.array([0, 5, 2]), np.ones(3))  # column 5 >= n_cols
    with pytest.raises(af.AfemError):
        af.applyNeumannToRhs(mesh, ls.rhsVariable(), np.array([[0, 1, 999999]]), 1.0, "value")


# ---------------------------------------------------------------- fallback kernels (high-valence nodes)
def fan_mesh_3d(m, seed=0):
    """A node (0) with 2m incident tetrahedra: a ring of m nodes around it, two
    apexes; row 0 has m + 3 non-zeros."""
    rng = np.random.default_rng(seed)
    ang = 2 * np.pi * (np.arange(m) + 0.3 * rng.random(m)) / m
    ring = np.c_[np.cos(ang), np.sin(ang), 0.1 * rng.standard_normal(m)]
    coords = np.vstack([[0.0, 0.0, 0.0], ring, [0.05, -0.02, 1.0], [-0.03, 0.04, -1.0]])
    top, bot = m + 1, m + 2
    cells = []
    for i in range(m):
        a, b = 1 + i, 1 + (i + 1) % m
        cells.append([0, a, b, top])
        cells.append([0, b, a, bot])
    return np.array(cells, dtype=np.int32), coords


def fan_mesh_2d(m, seed=0):
    rng = np.random.default_rng(seed)
    ang = 2 * np.pi * (np.arange(m) + 0.3 * rng.random(m)) / m
    r = 1.0 + 0.1 * rng.random(m)
    coords = np.vstack([[0.0, 0.0, 0.0], np.c_[r * np.cos(ang), r * np.sin(ang), np.zeros(m)]])
    cells = [[0, 1 + i, 1 + (i + 1) % m] for i in range(m)]
    return np.array(cells, dtype=np.int32), coords


@pytest.mark.parametrize("dim,m,kern", [(3, 32, K_TILE), (3, 40, K_GLOBAL), (2, 100, K_GLOBAL), (3, 12, K_STRIP)])
def test_fan_mesh_scalar_fallbacks(ctx, dim, m, kern):
    cells, coords = fan_mesh_3d(m) if dim == 3 else fan_mesh_2d(m)
    n = coords.shape[0]
    mesh = af.Mesh.from_arrays(ctx, dim, cells, coords)
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    bsr.computeSparsity()
    ls = af.DoFLinearSystem().initialize(ctx, n)
    bsr.assemblePoissonP1(1.0, 3.0, ls.rhsVariable())
    assert bsr.stats()["last_kernel"] == kern
    rows, cols, vals = bsr.download()
    orp, ocols = O.sparsity(n, n, cells)
    ovals, orhs = O.assemble_poisson(n, cells, coords, orp, ocols, 3.0)
    assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
    _close(vals, ovals)
    _close(ls.rhs_host(), orhs)
    # and the RHS accumulates on the fallbacks too
    bsr.assemblePoissonP1(1.0, 3.0, ls.rhsVariable())
    _close(ls.rhs_host(), 2 * orhs)


@pytest.mark.parametrize("m,kern,env", [(40, K_E3_GLOBAL, None), (31, K_E3_GLOBAL, None), (12, K_E3_WG, None),
                                        (12, K_E3_STRIP, "AFEM_ELAST_WG"), (12, K_E3_ITEM, "AFEM_ELAST_STRIP")])
@pytest.mark.parametrize("use_csr", [False, True])
def test_fan_mesh_block3_fallback(ctx, variant, m, kern, env, use_csr):
    if env:  # the alternative kernels, forced
        variant("AFEM_ELAST_WG", "0")
        variant(env, "0")
    cells, coords = fan_mesh_3d(m, seed=2)
    n = coords.shape[0]
    mesh = af.Mesh.from_arrays(ctx, 3, cells, coords)
    bsr = af.BSRFormat(mesh, 3).initialize(use_csr)
    bsr.computeSparsity()
    d = ctx.malloc(8 * 3 * n)
    bsr.assembleElasticityP1Ex(1.2e5, 1.6e5, 2.5e3, (0.5, -1.0, 2.0), d, rhs_mode="set")
    assert bsr.stats()["last_kernel"] == kern
    rows, cols, vals = bsr.download()
    rhs = ctx.to_host(d, 3 * n, np.float64)
    ctx.free(d)
    orp, ocols = O.sparsity(n, n, cells)
    ovals, orhs = O.assemble_elasticity_tet(n, cells, coords, orp, ocols, 1.2e5, 1.6e5, 2.5e3, (0.5, -1.0, 2.0))
    if use_csr:
        ovals = O.blocks_to_row_order_k(orp, ovals, 3)
    assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
    _close(vals, ovals)
    _close(rhs, orhs)


def test_fan_mesh_block2(ctx):
    cells, coords = fan_mesh_2d(90, seed=4)
    n = coords.shape[0]
    mesh = af.Mesh.from_arrays(ctx, 2, cells, coords)
    for use_csr in (False, True):
        bsr = af.BSRFormat(mesh, 2).initialize(use_csr)
        bsr.computeSparsity()
        bsr.assembleElasticityP1(1.2e5, 1.6e5)
        rows, cols, vals = bsr.download()
        orp, ocols = O.sparsity(n, n, cells)
        ovals = O.assemble_elasticity_tri(n, cells, coords, orp, ocols, 1.2e5, 1.6e5)
        if use_csr:
            ovals = O.blocks_to_row_order(orp, ovals)
        _close(vals, ovals)


def test_apply_bcs_unsorted_view_and_row_tail(ctx):
    """k_apply_bcs (4 rows per thread, the diagonal of a forced row found by a
    binary search with a linear fallback): a host view whose rows are stored in
    a scrambled column order, a row count that is not a multiple of 4, forced
    and eliminated rows among the last ones -- the forced values land on the
    diagonals and the eliminated rows become identity rows, as the oracle's
    _applyForcedValuesToLhs / _applyRowElimination (HypreDoFLinearSystem.cc:319-382)."""
    gm = read_gmsh(path("circle_cut.msh"))
    n = gm.n_nodes
    orp, ocols = O.sparsity(n, n, gm.cells)
    ovals, orhs = O.assemble_poisson(n, gm.cells, gm.coords, orp, ocols, 5.5)
    rng = np.random.default_rng(11)
    cols, vals = ocols.copy(), ovals.copy()
    for r in range(n):  # every row's entries in a random order
        p = orp[r] + rng.permutation(orp[r + 1] - orp[r])
        cols[orp[r]:orp[r + 1]], vals[orp[r]:orp[r + 1]] = ocols[p], ovals[p]
    # the last rows (the partial group of 4 when n % 4 != 0) forced and eliminated; no row is
    # both (the reference eliminates first, then forces the diagonal: the oracle's order differs)
    forced = np.array([1, 2, n - 2, n - 1], dtype=np.int32)
    elim = np.array([3, n - 3], dtype=np.int32)
    ls = af.DoFLinearSystem().initialize(ctx, n)
    ls.setCSRValues(orp[:-1].astype(np.int32), np.diff(orp).astype(np.int32), cols, vals)
    ls.set_rhs_host(orhs)
    ls.applyDirichletViaPenalty(forced, 0.5, 1e30)
    ls.applyDirichletViaRowElimination(elim, 0.25)
    ls.applyBoundaryConditions()
    ov, orh = ovals.copy(), orhs.copy()
    O.dirichlet_penalty(forced, 0.5, 1e30, orp, ocols, ov, orh)
    O.row_elimination(elim, 0.25, orp, ocols, ov, orh)
    ls.setSolverOptions(method="direct")
    st = ls.solve()
    x = ls.solution_host()
    xo = np.linalg.solve(O.csr_to_dense(orp, ocols, ov), orh)
    assert st["converged"] and np.abs(x - xo).max() / np.abs(xo).max() <= SOL_TOL
    assert np.allclose(x[elim], 0.25) and np.allclose(x[forced], 0.5)


def test_assembly_ticket_ring_wraps(ctx, variant):
    """The persistent assembly kernels' claim counters come from a ring of 256
    per-assembly slots zeroed together (assembly.hip next_tickets): 300
    assemblies in a row (past a wrap) all give the same bits."""
    variant("AFEM_ASSEMBLY_CUBES", "0")  # the row-strip family (generator boxes default to cubes.hip)
    mesh = af.Mesh.structured(ctx, 3, 10, jitter=0.2, seed=3)
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    bsr.computeSparsity()
    ls = af.DoFLinearSystem().initialize(ctx, mesh.n_own_nodes)
    bsr.assemblePoissonP1(1.0, 2.0, ls.rhsVariable(), rhs_mode="set")
    _, _, ref = bsr.download()
    for i in range(300):
        bsr.assemblePoissonP1(1.0, 2.0, ls.rhsVariable(), rhs_mode="set")
        if i % 50 == 49 or i in (254, 255, 256, 257):
            _, _, v = bsr.download()
            assert np.array_equal(v, ref), i
