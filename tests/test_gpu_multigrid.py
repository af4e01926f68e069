"""Geometric multigrid preconditioner (afem_solver_opts.multigrid,
arcanefem_amd/csrc/multigrid.hip) on structured Kuhn boxes: the PCG with the
V-cycle reaches the oracle's direct solution (the same bar as the Jacobi-PCG,
tests/test_gpu_parity.py::test_structured_solve_parity), in far fewer
iterations; row elimination (non-symmetric rows) and meshes without a
structured grid (point-Jacobi fallback) keep working; the Newmark loop with the
reused hierarchy matches the oracle Newmark.

The reference's GPU solve is Hypre PCG + BoomerAMG
(femutils/HypreDoFLinearSystem.cc:387-762), an external library not present
here: only the solution is compared (parity of the preconditioner itself is
unpinned, as for the reference's own solver)."""
import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

import arcanefem_amd as af
from arcanefem_amd.gmsh import read_gmsh
from oracle import oracle as O

from golden_cases import path

pytestmark = pytest.mark.gpu

SOL_TOL = 1e-10
E, NU = 21e5, 0.28
LAM = E * NU / ((1 + NU) * (1 - 2 * NU))
MU2 = 2 * E / (2 * (1 + NU))


def _poisson(ctx, mesh, f=5.5):
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    bsr.computeSparsity()
    ls = af.DoFLinearSystem().initialize(ctx, mesh.n_own_nodes, mesh.n_nodes)
    bsr.assemblePoissonP1(1.0, f, ls.rhsVariable())
    bsr.toLinearSystem(ls)
    return bsr, ls


def _solve(ls, pc, rtol=1e-14):
    ls.setSolverOptions(rtol=rtol, max_iter=50000, method="pcg", preconditioner=pc)
    st = ls.solve()
    assert st["converged"], (pc, st)
    return ls.solution_host().copy(), st["iterations"]


@pytest.mark.parametrize("n", [8, 16])
def test_multigrid_poisson_matches_direct(ctx, n):
    mesh = af.Mesh.structured(ctx, 3, n)
    bsr, ls = _poisson(ctx, mesh)
    bottom = mesh.bottom_nodes()
    ls.applyDirichletViaPenalty(bottom, 0.5, 1e30)
    x_mg, it_mg = _solve(ls, "multigrid")
    x_j, it_j = _solve(ls, "jacobi")
    cells, coords, _ = mesh.download()
    orp, ocols = O.sparsity(mesh.n_nodes, mesh.n_own_nodes, cells)
    ovals, orhs = O.assemble_poisson(mesh.n_own_nodes, cells, coords, orp, ocols, 5.5)
    O.dirichlet_penalty(bottom, 0.5, 1e30, orp, ocols, ovals, orhs)
    xo = np.linalg.solve(O.csr_to_dense(orp, ocols, ovals), orhs)
    for x in (x_mg, x_j):
        assert np.abs(x - xo).max() / np.abs(xo).max() <= SOL_TOL
    assert it_mg <= 24 and 4 * it_mg <= it_j, (it_mg, it_j)


@pytest.mark.parametrize("use_csr", [False, True])
def test_multigrid_elasticity_matches_direct(ctx, use_csr):
    n = 12  # 12 -> 6 -> 3 cells: two coarse grids, the last (4^3 nodes, 192 DoF) inverted densely
    mesh = af.Mesh.structured(ctx, 3, n, seed=5)
    cells, coords, _ = mesh.download()
    bsr = af.BSRFormat(mesh, 3).initialize(use_csr)
    bsr.computeSparsity()
    ls = af.DoFLinearSystem().initialize(ctx, 3 * mesh.n_own_nodes, 3 * mesh.n_nodes)
    bsr.assembleElasticityP1Ex(LAM, MU2, 0.0, (0.0, 0.0, -1.0), ls.rhsVariable(), rhs_mode="set")
    bsr.toLinearSystem(ls)
    fixed = np.arange(2 * (n + 1) ** 2)  # the two bottom node layers clamped
    dofs = (3 * fixed[:, None] + np.arange(3)[None, :]).ravel().astype(np.int32)
    ls.applyDirichletViaPenalty(dofs, 0.0, 1e30)
    x_mg, it_mg = _solve(ls, "multigrid", rtol=1e-13)
    x_j, it_j = _solve(ls, "jacobi", rtol=1e-13)
    nn = mesh.n_own_nodes
    rp, cols = O.sparsity(mesh.n_nodes, nn, cells)
    vals, rhs = O.assemble_elasticity_tet(nn, cells, coords, rp, cols, LAM, MU2, 0.0, (0.0, 0.0, -1.0))
    blk_row = np.repeat(np.arange(nn), np.diff(rp))
    ii = (3 * blk_row[:, None, None] + np.arange(3)[None, :, None] + 0 * np.arange(3)[None, None, :]).ravel()
    jj = (3 * cols[:, None, None] + 0 * np.arange(3)[None, :, None] + np.arange(3)[None, None, :]).ravel()
    A = sp.csr_matrix((vals, (ii, jj)), shape=(3 * nn, 3 * nn)).tolil()
    for d in dofs:
        A[d, d] = 1e30
    rhs[dofs] = 0.0
    xo = spla.spsolve(A.tocsc(), rhs)
    for x in (x_mg, x_j):
        assert np.abs(x - xo).max() <= 1e-8 * np.abs(xo).max()
    assert 4 * it_mg <= it_j, (it_mg, it_j)


def test_multigrid_fp32_cycle_products(ctx, variant):
    """Block-3 multigrid with the cycle's products on fp32 copies (AFEM_MG_F32:
    0 none, 1 the fine level, 2 every level -- the default) and the fused entry
    / exit (AFEM_MG_FUSE): the PCG's own product stays fp64, so every variant
    reaches the same solution at the tolerance (the oracle's direct solve) in
    about the same iterations; the fused entry / exit gives the bits of the
    separate passes."""
    n = 16  # 16 -> 8 -> 4 cells: two coarse grids
    mesh = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=7)
    cells, coords, _ = mesh.download()
    bsr = af.BSRFormat(mesh, 3).initialize(True)
    bsr.computeSparsity()
    ls = af.DoFLinearSystem().initialize(ctx, 3 * mesh.n_own_nodes, 3 * mesh.n_nodes)
    bsr.assembleElasticityP1Ex(LAM, MU2, 0.0, (0.0, 0.0, -1.0), ls.rhsVariable(), rhs_mode="set")
    bsr.toLinearSystem(ls)
    fixed = np.arange((n + 1) ** 2)  # the bottom node layer clamped
    dofs = (3 * fixed[:, None] + np.arange(3)[None, :]).ravel().astype(np.int32)
    xs, its = {}, {}
    for f32, fuse in (("0", "0"), ("1", "1"), ("2", "0"), ("2", "1")):
        variant("AFEM_MG_F32", f32)
        variant("AFEM_MG_FUSE", fuse)
        ls.applyDirichletViaPenalty(dofs, 0.0, 1e30)
        xs[f32 + fuse], its[f32 + fuse] = _solve(ls, "multigrid", rtol=1e-12)
    nn = mesh.n_own_nodes
    rp, cols = O.sparsity(mesh.n_nodes, nn, cells)
    vals, rhs = O.assemble_elasticity_tet(nn, cells, coords, rp, cols, LAM, MU2, 0.0, (0.0, 0.0, -1.0))
    blk_row = np.repeat(np.arange(nn), np.diff(rp))
    ii = (3 * blk_row[:, None, None] + np.arange(3)[None, :, None] + 0 * np.arange(3)[None, None, :]).ravel()
    jj = (3 * cols[:, None, None] + 0 * np.arange(3)[None, :, None] + np.arange(3)[None, None, :]).ravel()
    A = sp.csr_matrix((vals, (ii, jj)), shape=(3 * nn, 3 * nn)).tolil()
    for d in dofs:
        A[d, d] = 1e30
    rhs[dofs] = 0.0
    xo = spla.spsolve(A.tocsc(), rhs)
    print(f"multigrid fp32 variants: iterations {its}")
    for k, x in xs.items():
        assert np.abs(x - xo).max() <= 1e-8 * np.abs(xo).max(), k
        assert abs(its[k] - its["00"]) <= 2, its
    # the fused entry / exit: the same bits as the separate passes
    assert np.array_equal(xs["20"], xs["21"]) and its["20"] == its["21"]


def test_multigrid_penalty_beyond_fp32(ctx):
    """Block-3 multigrid with a penalty above the fp32 range (1e40): the fp32
    cycle copies saturate it and the PCG reaches the Jacobi-PCG's solution."""
    n = 8
    mesh = af.Mesh.structured(ctx, 3, n, seed=3)
    bsr = af.BSRFormat(mesh, 3).initialize(True)
    bsr.computeSparsity()
    ls = af.DoFLinearSystem().initialize(ctx, 3 * mesh.n_own_nodes, 3 * mesh.n_nodes)
    bsr.assembleElasticityP1Ex(LAM, MU2, 0.0, (0.0, 0.0, -1.0), ls.rhsVariable(), rhs_mode="set")
    bsr.toLinearSystem(ls)
    fixed = np.arange((n + 1) ** 2)
    dofs = (3 * fixed[:, None] + np.arange(3)[None, :]).ravel().astype(np.int32)
    ls.applyDirichletViaPenalty(dofs, 0.0, 1e40)
    x_mg, _ = _solve(ls, "multigrid", rtol=1e-12)
    ls.applyDirichletViaPenalty(dofs, 0.0, 1e40)
    x_j, _ = _solve(ls, "jacobi", rtol=1e-12)
    assert np.isfinite(x_mg).all()
    assert np.abs(x_mg - x_j).max() <= 1e-8 * np.abs(x_j).max()


def test_multigrid_row_elimination(ctx):
    # eliminated rows (identity rows, columns kept: a non-symmetric matrix) stay
    # out of the V-cycle: same solution as the Jacobi-PCG
    mesh = af.Mesh.structured(ctx, 3, 16)
    bsr, ls = _poisson(ctx, mesh)
    ls.applyDirichletViaRowElimination(mesh.bottom_nodes(), 0.5)
    x_j, _ = _solve(ls, "jacobi")
    x_mg, it_mg = _solve(ls, "multigrid")
    assert np.abs(x_mg - x_j).max() / np.abs(x_j).max() <= SOL_TOL
    assert it_mg <= 30


def test_multigrid_reuse_and_rebuild(ctx):
    # "multigrid-reuse" keeps the hierarchy of the first solve: a re-assembled
    # matrix with other values (here: 3x the coefficient) still converges to
    # its own solution (stale coarse operators only slow the iteration)
    mesh = af.Mesh.structured(ctx, 3, 16)
    bsr, ls = _poisson(ctx, mesh)
    bottom = mesh.bottom_nodes()
    ls.applyDirichletViaPenalty(bottom, 0.5, 1e30)
    x1, _ = _solve(ls, "multigrid-reuse")
    bsr.assemblePoissonP1(3.0, 5.5, ls.rhsVariable(), rhs_mode="set")
    bsr.toLinearSystem(ls)
    ls.applyDirichletViaPenalty(bottom, 0.5, 1e30)
    x2, it2 = _solve(ls, "multigrid-reuse")
    x3, _ = _solve(ls, "jacobi")
    assert np.abs(x2 - x3).max() / np.abs(x3).max() <= SOL_TOL
    assert not np.allclose(x1, x2)


@pytest.mark.parametrize("which", ["sphere", "odd"])
def test_multigrid_falls_back_to_jacobi(ctx, which):
    # no structured grid (Gmsh mesh) or no coarse grid (odd cell count): the
    # multigrid option runs the point-Jacobi PCG
    if which == "sphere":
        gm = read_gmsh(path("sphere_cut.msh"))
        mesh = af.Mesh.from_arrays(ctx, 3, gm.cells, gm.coords)
        dir_nodes = gm.group_nodes("horizontal").astype(np.int32)
    else:
        mesh = af.Mesh.structured(ctx, 3, 9)
        dir_nodes = mesh.bottom_nodes()
    bsr, ls = _poisson(ctx, mesh)
    ls.applyDirichletViaPenalty(dir_nodes, 0.5, 1e30)
    x_j, it_j = _solve(ls, "jacobi")
    x_mg, it_mg = _solve(ls, "multigrid")
    assert it_mg == it_j and np.array_equal(x_mg, x_j)


def test_multigrid_option_validation(ctx):
    mesh = af.Mesh.structured(ctx, 3, 4)
    bsr = af.BSRFormat(mesh, 3).initialize(True)
    bsr.computeSparsity()
    ls = af.DoFLinearSystem().initialize(ctx, 3 * mesh.n_own_nodes)
    o = af._capi.SolverOpts()
    af._capi.call("afem_ls_get_solver_options", ls.impl, af._capi.ctypes.byref(o))
    o.multigrid = 3
    with pytest.raises(af.AfemError):
        af._capi.call("afem_ls_set_solver_options", ls.impl, af._capi.ctypes.byref(o))
    o.multigrid, o.precond_block = 1, 3
    with pytest.raises(af.AfemError):
        af._capi.call("afem_ls_set_solver_options", ls.impl, af._capi.ctypes.byref(o))


def test_elastodynamics_multigrid_matches_oracle(ctx):
    # C5 semantics (as test_gpu_elasticity3d.py::test_elastodynamics_newmark_parity)
    # with the multigrid hierarchy built at the first step and reused
    from arcanefem_amd.elastodynamics import Elastodynamics3D

    n = 8
    mesh = af.Mesh.structured(ctx, 3, n)
    cells, coords, _ = mesh.download()
    ids = np.arange(mesh.n_own_nodes)
    fixed = ids[ids % (n + 1) == 0]  # node x-index 0
    E_, nu_, rho, dt = 21e5, 0.28, 1.0, 1e-3
    f = (0.0, -9.81, 1.0)
    res = {}
    for pc in ("multigrid", "jacobi"):
        sim = Elastodynamics3D(ctx, mesh, E_, nu_, rho, dt, body_force=f, fixed_nodes=fixed, rtol=1e-13,
                               preconditioner=pc)
        its = []
        for _ in range(4):
            st = sim.step()
            assert st["converged"]
            its.append(st["iterations"])
        res[pc] = (sim.state_host(), its)
        sim.close()
    Uo, Vo, Ao = O.newmark_elastodynamics(mesh.n_nodes, cells, coords, E_, nu_, rho, dt, 4, f, fixed)
    for g, o in zip(res["multigrid"][0], (Uo, Vo, Ao)):
        assert np.abs(g - o).max() <= 1e-8 * np.abs(o).max(), np.abs(g - o).max() / np.abs(o).max()
    assert max(res["multigrid"][1]) * 3 <= min(res["jacobi"][1]), (res["multigrid"][1], res["jacobi"][1])
