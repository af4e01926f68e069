"""Block-3 P1 elasticity on tetrahedra (BASELINE config C3) and its Newmark
LHS form c0*M + K (config C5): the HIP kernel through the C ABI against the
oracle's restatement (oracle/oracle.c orc_assemble_elasticity_tet).

Parity is against the oracle restatement (the reference's 2D element,
modules/elasticity/FemModule.h:112-140, in 3D), which is pinned by the
reference's own 3D case: passmo's Gauss-point element equals it to 1e-13 and
its Newmark replay meets the bar3d-tetra golden (tests/test_oracle_passmo.py;
the same replay through libafem: tests/test_gpu_passmo.py), plus the known
answers of tests/test_oracle_elasticity3d.py.
Tolerance: |gpu - oracle| <= 1e-12 * max|oracle| per entry.
"""
import numpy as np
import pytest

import arcanefem_amd as af
from arcanefem_amd.gmsh import read_gmsh
from oracle import oracle as O

from golden_cases import path

pytestmark = pytest.mark.gpu

VAL_TOL = 1e-12
E, NU = 21e5, 0.28
LAM = E * NU / ((1 + NU) * (1 - 2 * NU))
MU2 = 2 * E / (2 * (1 + NU))


def _mesh(ctx, which):
    if which == "box":
        return af.Mesh.structured(ctx, 3, 6)
    if which == "bigbox":  # interior 4x4x4 bricks: the uniform-strip instance runs
        return af.Mesh.structured(ctx, 3, 13, seed=5)
    if which == "sphere":
        gm = read_gmsh(path("sphere_cut.msh"))
        return af.Mesh.from_arrays(ctx, 3, gm.cells, gm.coords)
    if which == "lshape":
        gm = read_gmsh(path("L-shape-3D.msh"))
        return af.Mesh.from_arrays(ctx, 3, gm.cells, gm.coords)
    return af.Mesh.structured(ctx, 3, 5, nz=9, nranks=3, rank=1)


@pytest.mark.parametrize("which", ["box", "bigbox", "sphere", "lshape", "slab"])
@pytest.mark.parametrize("use_csr", [False, True])
@pytest.mark.parametrize("c0,force", [(0.0, None), (3.7e6, (0.5, -1.0, 2.0))])
def test_elasticity3d_assembly_parity(ctx, which, use_csr, c0, force):
    mesh = _mesh(ctx, which)
    bsr = af.BSRFormat(mesh, 3).initialize(use_csr)
    bsr.computeSparsity()
    n3 = 3 * mesh.n_own_nodes
    drhs = ctx.malloc(8 * n3)
    ctx.to_device(drhs, np.zeros(n3))
    bsr.assembleElasticityP1Ex(LAM, MU2, c0, force, drhs if force else None)
    rows, cols, vals = bsr.download()
    rhs = ctx.to_host(drhs, n3, np.float64)
    ctx.free(drhs)
    cells, coords, _ = mesh.download()
    orp, ocols = O.sparsity(mesh.n_nodes, mesh.n_own_nodes, cells)
    ovals, orhs = O.assemble_elasticity_tet(mesh.n_own_nodes, cells, coords, orp, ocols, LAM, MU2, c0, force)
    if use_csr:
        ovals = O.blocks_to_row_order_k(orp, ovals, 3)
    assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
    err = np.abs(vals - ovals).max() / np.abs(ovals).max()
    assert err <= VAL_TOL, f"block-3 values differ from the oracle: {err:.3e}"
    if force:
        assert np.abs(rhs - orhs).max() <= VAL_TOL * np.abs(orhs).max()


@pytest.mark.parametrize("use_csr", [False, True])
def test_elasticity3d_uniform_variant_bitwise(ctx, variant, use_csr):
    mesh = _mesh(ctx, "bigbox")
    bsr = af.BSRFormat(mesh, 3).initialize(use_csr)
    bsr.computeSparsity()
    assert bsr.stats()["uniform_slices"] > 0
    n3 = 3 * mesh.n_own_nodes
    drhs = ctx.malloc(8 * n3)
    bsr.assembleElasticityP1Ex(LAM, MU2, 3.7e6, (0.5, -1.0, 2.0), drhs, rhs_mode="set")
    v_uni, r_uni = bsr.download()[2], ctx.to_host(drhs, n3, np.float64)
    variant("AFEM_ASSEMBLY_UNIFORM", "0")
    bsr.assembleElasticityP1Ex(LAM, MU2, 3.7e6, (0.5, -1.0, 2.0), drhs, rhs_mode="set")
    v_gen, r_gen = bsr.download()[2], ctx.to_host(drhs, n3, np.float64)
    ctx.free(drhs)
    assert np.array_equal(v_uni, v_gen), "uniform and general block-3 instances differ"
    assert np.array_equal(r_uni, r_gen)


def test_elasticity3d_box_edges_stay_on_the_workgroup_kernel(ctx, variant):
    """A box whose edges hold full runs (boundary-aware order: 32 rows per edge
    slice) still fits the block-3 workgroup kernel (slices <= 256 nodes), and
    its uniform / general instances give the same bits."""
    mesh = af.Mesh.structured(ctx, 3, 70, jitter=0.2, seed=9)
    bsr = af.BSRFormat(mesh, 3).initialize(False)
    bsr.computeSparsity()
    st = bsr.stats()
    assert st["max_slice_nodes"] <= 256, st
    n3 = 3 * mesh.n_own_nodes
    drhs = ctx.malloc(8 * n3)
    bsr.assembleElasticityP1Ex(LAM, MU2, 3.7e6, (0.5, -1.0, 2.0), drhs, rhs_mode="set")
    assert bsr.stats()["last_kernel"] == 8
    v_k, r_k = bsr.download()[2], ctx.to_host(drhs, n3, np.float64)
    variant("AFEM_ASSEMBLY_UNIFORM", "0")
    bsr.assembleElasticityP1Ex(LAM, MU2, 3.7e6, (0.5, -1.0, 2.0), drhs, rhs_mode="set")
    v_g, r_g = bsr.download()[2], ctx.to_host(drhs, n3, np.float64)
    ctx.free(drhs)
    assert np.array_equal(v_k, v_g) and np.array_equal(r_k, r_g)


@pytest.mark.parametrize("n", [13, 22])
@pytest.mark.parametrize("use_csr", [False, True])
def test_elasticity3d_stencil_instance_bitwise(ctx, variant, n, use_csr):
    """Interior bricks (compiled-in signature 0) run the workgroup kernel's
    stencil instance (step bytes and shift/swap arms as constants): the same
    bits as the uniform instance (AFEM_ASSEMBLY_STENCIL=0) and the oracle's
    values."""
    mesh = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=4)
    bsr = af.BSRFormat(mesh, 3).initialize(use_csr)
    bsr.computeSparsity()
    st = bsr.stats()
    assert st["stencil_sig"] == 0 and st["stencil_slices"] > 0
    n3 = 3 * mesh.n_own_nodes
    drhs = ctx.malloc(8 * n3)
    bsr.assembleElasticityP1Ex(LAM, MU2, 3.7e6, (0.5, -1.0, 2.0), drhs, rhs_mode="set")
    assert bsr.stats()["last_kernel"] == 8
    v_k, r_k = bsr.download()[2], ctx.to_host(drhs, n3, np.float64)
    variant("AFEM_ASSEMBLY_STENCIL", "0")
    bsr.assembleElasticityP1Ex(LAM, MU2, 3.7e6, (0.5, -1.0, 2.0), drhs, rhs_mode="set")
    rows, cols, v_u = bsr.download()
    r_u = ctx.to_host(drhs, n3, np.float64)
    ctx.free(drhs)
    assert np.array_equal(v_k, v_u), f"{np.count_nonzero(v_k != v_u)} values differ"
    assert np.array_equal(r_k, r_u)
    cells, coords, _ = mesh.download()
    orp, ocols = O.sparsity(mesh.n_nodes, mesh.n_own_nodes, cells)
    ovals, orhs = O.assemble_elasticity_tet(mesh.n_own_nodes, cells, coords, orp, ocols, LAM, MU2, 3.7e6,
                                            (0.5, -1.0, 2.0))
    if use_csr:
        ovals = O.blocks_to_row_order_k(orp, ovals, 3)
    assert np.abs(v_k - ovals).max() <= VAL_TOL * np.abs(ovals).max()
    assert np.abs(r_k - orhs).max() <= VAL_TOL * np.abs(orhs).max()


@pytest.mark.parametrize("which", ["bigbox", "box"])
@pytest.mark.parametrize("use_csr", [False, True])
def test_elasticity3d_workgroup_kernel_bitwise(ctx, variant, which, use_csr):
    """The three-wave-per-slice kernel (k_assemble_elast_wg) against the
    one-wave-per-(slice, component) kernel: the same arithmetic per entry (up
    to the compiler's FMA contraction: last-bit differences)."""
    mesh = _mesh(ctx, which)
    bsr = af.BSRFormat(mesh, 3).initialize(use_csr)
    bsr.computeSparsity()
    n3 = 3 * mesh.n_own_nodes
    drhs = ctx.malloc(8 * n3)
    bsr.assembleElasticityP1Ex(LAM, MU2, 3.7e6, (0.5, -1.0, 2.0), drhs, rhs_mode="set")
    assert bsr.stats()["last_kernel"] == 8
    v_wg, r_wg = bsr.download()[2], ctx.to_host(drhs, n3, np.float64)
    variant("AFEM_ELAST_WG", "0")
    bsr.assembleElasticityP1Ex(LAM, MU2, 3.7e6, (0.5, -1.0, 2.0), drhs, rhs_mode="set")
    assert bsr.stats()["last_kernel"] == 4
    v_st, r_st = bsr.download()[2], ctx.to_host(drhs, n3, np.float64)
    ctx.free(drhs)
    dv = np.abs(v_wg - v_st).max() / np.abs(v_st).max()
    dr = np.abs(r_wg - r_st).max() / np.abs(r_st).max()
    print(f"wg vs strip: values max rel {dv:.2e} ({np.count_nonzero(v_wg != v_st)} of {v_st.size} differ), rhs {dr:.2e}")
    # the same formulas; the compiler's FMA contraction may differ by kernel (last-bit differences)
    assert dv <= 1e-15 and dr <= 1e-15


@pytest.mark.parametrize("levels", [2, 3])
@pytest.mark.parametrize("use_csr", [False, True])
def test_elasticity3d_unstructured_refined(ctx, variant, levels, use_csr):
    """An unstructured mesh (the reference's L-shape-3D refined `levels` times:
    irregular valences, rows longer than 16, Hilbert slices beyond 256 nodes at
    3 levels) through the block-3 kernel for such meshes (AFEM_KERNEL_ELAST3_BIG)
    against the oracle, and against the global-memory kernel."""
    import bench

    gm = read_gmsh(path("L-shape-3D.msh"))
    cells, coords = bench.refine_tets(gm.cells, gm.coords, levels, "cpu")
    mesh = af.Mesh.from_arrays(ctx, 3, cells, coords)
    bsr = af.BSRFormat(mesh, 3).initialize(use_csr)
    bsr.computeSparsity()
    n = mesh.n_own_nodes
    drhs = ctx.malloc(8 * 3 * n)
    bsr.assembleElasticityP1Ex(LAM, MU2, 3.7e6, (0.5, -1.0, 2.0), drhs, rhs_mode="set")
    st = bsr.stats()
    print("max_slice_width", st["max_slice_width"], "max_slice_nodes", st["max_slice_nodes"], "kernel",
          st["last_kernel"])
    assert st["last_kernel"] in (8, 9)
    rows, cols, vals = bsr.download()
    rhs = ctx.to_host(drhs, 3 * n, np.float64)
    orp, ocols = O.sparsity(n, n, cells)
    ovals, orhs = O.assemble_elasticity_tet(n, cells, coords, orp, ocols, LAM, MU2, 3.7e6, (0.5, -1.0, 2.0))
    if use_csr:
        ovals = O.blocks_to_row_order_k(orp, ovals, 3)
    assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
    assert np.abs(vals - ovals).max() <= VAL_TOL * np.abs(ovals).max()
    assert np.abs(rhs - orhs).max() <= VAL_TOL * np.abs(orhs).max()
    variant("AFEM_ELAST_BIG", "0")
    variant("AFEM_ELAST_WG", "0")
    variant("AFEM_ELAST_STRIP", "0")
    bsr.assembleElasticityP1Ex(LAM, MU2, 3.7e6, (0.5, -1.0, 2.0), drhs, rhs_mode="set")
    _, _, gvals = bsr.download()
    ctx.free(drhs)
    assert np.abs(vals - gvals).max() <= 1e-13 * np.abs(ovals).max()


def test_elasticity3d_plain_entry_point_equals_ex(ctx):
    mesh = af.Mesh.structured(ctx, 3, 4)
    b1 = af.BSRFormat(mesh, 3).initialize(False)
    b1.computeSparsity()
    b1.assembleElasticityP1(LAM, MU2)
    b2 = af.BSRFormat(mesh, 3).initialize(False)
    b2.computeSparsity()
    b2.assembleElasticityP1Ex(LAM, MU2, 0.0, None, None)
    assert np.array_equal(b1.download()[2], b2.download()[2])


def test_elasticity3d_rigid_modes_at_scale(ctx):
    # size-independent property (~330k DoF): the 6 rigid-body modes are in the
    # nullspace of the unconstrained stiffness; with the mass term, a rigid
    # translation gives M*1 whose sum is c0 * total volume
    mesh = af.Mesh.structured(ctx, 3, 47)
    bsr = af.BSRFormat(mesh, 3).initialize(False)
    bsr.computeSparsity()
    bsr.assembleElasticityP1(LAM, MU2)
    rows, cols, vals = bsr.download()
    cells, coords, _ = mesh.download()
    nb = rows.shape[0] - 1
    rid = np.repeat(np.arange(nb), np.diff(rows))
    blk = vals.reshape(-1, 3, 3)
    x = coords[:nb]
    scale = np.abs(vals).max()
    modes = []
    for d in range(3):
        u = np.zeros((x.shape[0], 3))
        u[:, d] = 1.0
        modes.append(u)
    for ax in range(3):
        w = np.zeros(3)
        w[ax] = 1.0
        modes.append(np.cross(w, x))
    for u in modes:
        r = np.zeros((nb, 3))
        np.add.at(r, rid, np.einsum("kij,kj->ki", blk, u[cols]))
        assert np.abs(r).max() <= 1e-10 * scale * np.abs(u).max()
    # symmetry of the block matrix: K[a,b] == K[b,a]^T
    key = rid.astype(np.int64) * nb + cols
    keyT = cols.astype(np.int64) * nb + rid
    order = np.argsort(key)
    posT = np.searchsorted(key[order], keyT)
    assert np.abs(blk - blk[order][posT].transpose(0, 2, 1)).max() <= 1e-13 * scale
    # mass: sum of M over all blocks of component 0 = c0 * volume (jittered box)
    b2 = af.BSRFormat(mesh, 3).initialize(False)
    b2.computeSparsity()
    b2.assembleElasticityP1Ex(0.0, 0.0, 2.0, None, None)
    m = b2.download()[2].reshape(-1, 3, 3)
    xc = coords[cells]
    vol = np.abs(np.linalg.det(np.stack([xc[:, 1] - xc[:, 0], xc[:, 2] - xc[:, 0], xc[:, 3] - xc[:, 0]], 1))).sum() / 6
    assert abs(m[:, 0, 0].sum() - 2.0 * vol) <= 1e-12 * vol
    assert np.abs(m[:, 0, 1]).max() == 0.0


def test_elastodynamics_newmark_parity(ctx):
    # config C5 semantics on a small box: 6 Newmark steps with per-step
    # re-assembly of c0 M + K, clamped x=0 face, gravity-like body force
    from arcanefem_amd.elastodynamics import Elastodynamics3D

    mesh = af.Mesh.structured(ctx, 3, 3)
    cells, coords, _ = mesh.download()
    fixed = np.nonzero(coords[:, 0] < 0.5 / 3)[0]  # the x = 0 node layer (jitter < h/2)
    assert fixed.size == 16
    E_, nu_, rho, dt = 21e5, 0.28, 1.0, 1e-3
    f = (0.0, -9.81, 1.0)
    sim = Elastodynamics3D(ctx, mesh, E_, nu_, rho, dt, body_force=f, fixed_nodes=fixed, rtol=1e-14)
    for _ in range(6):
        st = sim.step()
        assert st["converged"]
    U, V, A = sim.state_host()
    Uo, Vo, Ao = O.newmark_elastodynamics(mesh.n_nodes, cells, coords, E_, nu_, rho, dt, 6, f, fixed)
    for g, o in ((U, Uo), (V, Vo), (A, Ao)):
        assert np.abs(g - o).max() <= 1e-8 * np.abs(o).max(), np.abs(g - o).max() / np.abs(o).max()
    sim.close()


@pytest.mark.parametrize("kw", [dict(etam=0.3, etak=1e-3),
                                dict(time_discretization="generalized-alpha", alpm=0.2, alpf=0.4),
                                dict(time_discretization="generalized-alpha", alpm=0.2, alpf=0.4, etam=0.3,
                                     etak=1e-3)],
                         ids=["newmark-rayleigh", "alpha", "alpha-rayleigh"])
def test_elastodynamics_damping_and_alpha_parity(ctx, kw):
    """Rayleigh damping (etam, etak) and the generalized-alpha scheme
    (modules/elastodynamics/FemModule.cc:222-296, RHS :842-862): 6 steps on the
    C5-semantics box against the oracle's loop with the module's c0 .. c10."""
    from arcanefem_amd.elastodynamics import Elastodynamics3D

    mesh = af.Mesh.structured(ctx, 3, 3)
    cells, coords, _ = mesh.download()
    fixed = np.nonzero(coords[:, 0] < 0.5 / 3)[0]
    E_, nu_, rho, dt = 21e5, 0.28, 1.0, 1e-3
    f = (0.0, -9.81, 1.0)
    sim = Elastodynamics3D(ctx, mesh, E_, nu_, rho, dt, body_force=f, fixed_nodes=fixed, rtol=1e-14, **kw)
    for _ in range(6):
        assert sim.step()["converged"]
    U, V, A = sim.state_host()
    okw = dict(kw)
    if "time_discretization" in okw:
        okw["scheme"] = okw.pop("time_discretization")
    Uo, Vo, Ao = O.newmark_elastodynamics(mesh.n_nodes, cells, coords, E_, nu_, rho, dt, 6, f, fixed, **okw)
    for g, o in ((U, Uo), (V, Vo), (A, Ao)):
        assert np.abs(g - o).max() <= 1e-8 * np.abs(o).max(), np.abs(g - o).max() / np.abs(o).max()
    # the undamped Newmark run differs (the options are not ignored)
    sim0 = Elastodynamics3D(ctx, mesh, E_, nu_, rho, dt, body_force=f, fixed_nodes=fixed, rtol=1e-14)
    for _ in range(6):
        sim0.step()
    assert np.abs(sim0.state_host()[0] - U).max() > 1e-6 * np.abs(U).max()
    sim.close()
    sim0.close()


@pytest.mark.parametrize("which", ["sphere", "bigbox"])
def test_block_jacobi3_static_solve(ctx, which):
    """precond_block = 3 (3x3 node-block Jacobi): a clamped static elasticity
    solve reaches the oracle's direct solution like point Jacobi; penalty rows
    are decoupled from their block mates.  (Iteration counts are reported, not
    gated: on the Kuhn-box Newmark system of C5 block Jacobi takes more
    iterations than point Jacobi.)"""
    mesh = _mesh(ctx, which)
    cells, coords, _ = mesh.download()
    bsr = af.BSRFormat(mesh, 3).initialize(True)
    bsr.computeSparsity()
    ls = af.DoFLinearSystem().initialize(ctx, 3 * mesh.n_own_nodes, 3 * mesh.n_nodes)
    bsr.assembleElasticityP1Ex(LAM, MU2, 0.0, (0.0, 0.0, -1.0), ls.rhsVariable(), rhs_mode="set")
    bsr.toLinearSystem(ls)
    z = coords[:mesh.n_own_nodes, 2]
    fixed = np.nonzero(z <= z.min() + 0.15 * (z.max() - z.min()))[0]  # a clamped bottom slab
    dofs = (3 * fixed[:, None] + np.arange(3)[None, :]).ravel().astype(np.int32)
    ls.applyDirichletViaPenalty(dofs, 0.0, 1e30)
    xs, its = {}, {}
    for pc in ("jacobi", "block3"):
        ls.setSolverOptions(rtol=1e-13, max_iter=50000, method="pcg", preconditioner=pc)
        st = ls.solve()
        assert st["converged"], (pc, st)
        xs[pc], its[pc] = ls.solution_host(), st["iterations"]
    ls.setSolverOptions(preconditioner="jacobi")
    import scipy.sparse as sp
    import scipy.sparse.linalg as spla

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
    for pc in xs:
        assert np.abs(xs[pc] - xo).max() <= 1e-8 * np.abs(xo).max(), pc
    print("iterations", its)


def _blocks(rows, vals, k, use_csr):
    """[nnz_b, k, k] blocks of a BSR value array in either layout
    (femutils/BSRFormat.h:194-256: CSR order = per node row [i][s][j])."""
    if not use_csr:
        return vals.reshape(-1, k, k)
    out = np.empty((rows[-1], k, k))
    for r in range(rows.shape[0] - 1):
        a, b = rows[r], rows[r + 1]
        out[a:b] = vals[k * k * a:k * k * b].reshape(k, b - a, k).transpose(1, 0, 2)
    return out


@pytest.mark.parametrize("which", ["box", "slab", "lshape", "tri"])
@pytest.mark.parametrize("use_csr", [False, True])
@pytest.mark.parametrize("spmv", ["blk", "csr"])
def test_block_spmv_matches_block_product(ctx, variant, which, use_csr, spmv):
    # the node-block SpMV (k_spmv_blk: node columns instead of scalar ones)
    # and the scalar CSR kernels (AFEM_SPMV=v16) against the block product
    if spmv == "csr":
        variant("AFEM_SPMV", "v16")
    k = 2 if which == "tri" else 3
    mesh = af.Mesh.structured(ctx, 2, 21, seed=3) if which == "tri" else _mesh(ctx, which)
    bsr = af.BSRFormat(mesh, k).initialize(use_csr)
    bsr.computeSparsity()
    if k == 3:
        bsr.assembleElasticityP1Ex(LAM, MU2, 3.7e6, None, None)
    else:
        bsr.assembleElasticityP1(LAM, MU2)
    ls = af.DoFLinearSystem().initialize(ctx, k * mesh.n_own_nodes, k * mesh.n_nodes)
    bsr.toLinearSystem(ls)
    rows, cols, vals = bsr.download()
    x = np.random.default_rng(7).standard_normal(k * mesh.n_nodes)
    dx = ctx.malloc(x.nbytes)
    dy = ctx.malloc(8 * k * mesh.n_own_nodes)
    ctx.to_device(dx, x)
    ls.spmv(dx, dy)
    y = ctx.to_host(dy, k * mesh.n_own_nodes, np.float64)
    ctx.free(dx)
    ctx.free(dy)
    B = _blocks(rows, vals, k, use_csr)
    xb = x.reshape(-1, k)[cols]                          # [nnz_b, k]
    prod = np.einsum("sij,sj->si", B, xb)
    yo = np.zeros((rows.shape[0] - 1, k))
    np.add.at(yo, np.repeat(np.arange(rows.shape[0] - 1), np.diff(rows)), prod)
    assert np.abs(y - yo.ravel()).max() <= 1e-13 * np.abs(yo).max()


# ---------------------------------------------------------------- C3 at its own size
def _kuhn_neighbourhood(n, g, seed=20250220, jitter=0.2):
    """The (up to 8) cubes around global node g of the generator's n^3 Kuhn
    box with their exact coordinates: local cells, node ids, coordinates."""
    np1 = n + 1
    i, j, k = g % np1, (g // np1) % np1, g // (np1 * np1)
    cubes = [(a, b, c) for a in (i - 1, i) for b in (j - 1, j) for c in (k - 1, k)
             if 0 <= a < n and 0 <= b < n and 0 <= c < n]
    e = np.eye(3, dtype=np.int64)
    tets = []
    for cube in cubes:
        v0 = np.array(cube)
        for perm in O.KUHN_PERMS:
            v1 = v0 + e[perm[0]]
            v2 = v1 + e[perm[1]]
            tets.append([v0, v1, v2, v0 + 1])
    T = np.array(tets)
    gid = T[..., 0] + np1 * (T[..., 1] + np1 * T[..., 2])
    nodes, local = np.unique(gid, return_inverse=True)
    local = local.reshape(gid.shape).astype(np.int32)
    h = 1.0 / n
    ijk = np.stack([nodes % np1, (nodes // np1) % np1, nodes // (np1 * np1)], 1)
    xyz = np.zeros((nodes.shape[0], 3))
    for c in range(3):
        u = O.hash_u01(seed, nodes * 3 + c)
        xyz[:, c] = ijk[:, c].astype(np.float64) * h + (u - 0.5) * (jitter * h)
    return nodes, local, xyz


def test_c3_full_size_properties(ctx):
    """BASELINE config C3 at its own size (n = 170: 5.0 M nodes, 15.0 M DoF,
    74.3 M blocks, per-block layout as the bench's c3 leg): the structure size
    nnz_b = 2E + N; the six rigid-body modes (3 translations, 3 rotations
    x -> w x x, exact in P1) in the kernel of K through the product SpMV;
    on ~400 sampled rows the block row against the oracle's
    (orc_assemble_elasticity_tet on the row's cube neighbourhood with the
    generator's exact coordinates) per entry at 1e-12 of the row's largest
    entry, and block symmetry K_cr = K_rc^T; the body-force total f x volume."""
    n = 170
    mesh = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=20250220)
    N = mesh.n_own_nodes
    assert N == (n + 1) ** 3
    bsr = af.BSRFormat(mesh, 3).initialize(False)
    bsr.computeSparsity()
    n3 = 3 * N
    drhs = ctx.malloc(8 * n3)
    bsr.assembleElasticityP1Ex(LAM, MU2, 0.0, (0.0, 0.0, -1.0), drhs, rhs_mode="set")
    rhs = ctx.to_host(drhs, n3, np.float64)
    ctx.free(drhs)
    nnz_b = bsr.view().nnz_blocks
    edges = 3 * n * (n + 1) ** 2 + 3 * n * n * (n + 1) + n ** 3
    assert nnz_b == 2 * edges + N
    rows, cols, vals = bsr.download()
    vmax = np.abs(vals).max()
    _, coords, _ = mesh.download()
    # rigid-body modes through the product SpMV (k_spmv_blk on the node-row structure)
    ls = af.DoFLinearSystem().initialize(ctx, n3)
    bsr.toLinearSystem(ls)
    x = ctx.malloc(8 * n3)
    y = ctx.malloc(8 * n3)
    X = coords[:N]
    modes = []
    for a in range(3):
        v = np.zeros((N, 3))
        v[:, a] = 1.0
        modes.append(v)
    for w in np.eye(3):
        modes.append(np.cross(w, X))
    worst = 0.0
    for v in modes:
        ctx.to_device(x, v.ravel())
        ls.spmv(x, y)
        r = ctx.to_host(y, n3, np.float64)
        worst = max(worst, np.abs(r).max() / (vmax * np.abs(v).max()))
    ctx.free(x)
    ctx.free(y)
    assert worst <= 1e-12, worst
    # sampled rows: oracle parity per entry and block symmetry
    rng = np.random.default_rng(170)
    samples = np.concatenate([rng.integers(0, N, 400), [0, N - 1, (n + 1) ** 2 * 85 + (n + 1) * 5 + 3]])
    worst_row = 0.0
    for g in samples:
        s, e = int(rows[g]), int(rows[g + 1])
        nodes, local, xyz = _kuhn_neighbourhood(n, int(g))
        orp, ocols = O.sparsity(nodes.shape[0], nodes.shape[0], local)
        ov, _ = O.assemble_elasticity_tet(nodes.shape[0], local, xyz, orp, ocols, LAM, MU2)
        rl = int(np.searchsorted(nodes, g))
        assert np.array_equal(cols[s:e], nodes[ocols[orp[rl]:orp[rl + 1]]])
        orow = ov[9 * orp[rl]:9 * orp[rl + 1]]
        grow = vals[9 * s:9 * e]
        worst_row = max(worst_row, np.abs(grow - orow).max() / np.abs(orow).max())
        for t in range(s, e):
            c = int(cols[t])
            tt = int(rows[c]) + int(np.searchsorted(cols[rows[c]:rows[c + 1]], g))
            assert cols[tt] == g
            bt = vals[9 * tt:9 * tt + 9].reshape(3, 3)
            assert np.abs(bt.T - vals[9 * t:9 * t + 9].reshape(3, 3)).max() <= 1e-14 * vmax
    assert worst_row <= VAL_TOL, worst_row
    # the body force's total: f_z x volume of the (jitter-deformed) unit box
    assert abs(rhs[2::3].sum() + 1.0) < 1e-3 and abs(rhs[0::3].sum()) < 1e-12
    print(f"C3 n={n}: {n3} DoF, {nnz_b} blocks; rigid modes max |K v| / (max|K| max|v|) {worst:.2e}; "
          f"sampled rows max rel {worst_row:.2e}")
    ls.reset()
    bsr.close()
    mesh.close()


def test_c5_full_size_properties(ctx):
    """BASELINE config C5's per-step operator at the bench's size (n = 128:
    2.15 M nodes, 6.45 M DoF), after Newmark steps with the
    multigrid PCG (modules/passmo/ElastodynamicModule.cc:469-536 re-assembles
    it every step): the re-assembled c0 M + K(c1, c2) read back through
    afem_elastodynamics_operators --
      * c0 = rho / (beta dt^2) and c1, c2 = lambda, 2 mu (FemModule.cc:255-264);
      * symmetry on sampled scalar rows;
      * the stiffness part lhs - c0 M has the six rigid-body modes in its kernel
        on every unclamped row (orc_spmv on the host), and the clamped rows
        carry the penalty diagonal;
      * the consistent mass sums to 3 x volume (unit density; rho is in c0);
      * sampled block rows equal the oracle's (orc_assemble_elasticity_tet with
        c0 on the row's cube neighbourhood, generator coordinates) to 1e-12 of
        the row's largest entry;
      * every step converged, displacements finite and downward."""
    from arcanefem_amd.elastodynamics import Elastodynamics3D

    n = 128
    mesh = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=20250220)
    N = mesh.n_own_nodes
    ids = np.arange(N)
    fixed = ids[ids % (n + 1) == 0].astype(np.int32)
    rho, dt = 2.5, 1e-3
    dyn = Elastodynamics3D(ctx, mesh, E, NU, rho, dt, body_force=(0.0, 0.0, -1.0), fixed_nodes=fixed, rtol=1e-8,
                           preconditioner="multigrid")
    for _ in range(3):
        st = dyn.step()
        assert st["converged"], st
    U = dyn.state_host()[0]
    assert np.isfinite(U).all() and U[2::3].sum() < 0
    ops = dyn.operators()
    v, c = ops["lhs"], ops["c"]
    beta = 0.25
    assert abs(c[0] - rho / (beta * dt * dt)) <= 1e-12 * c[0]
    assert abs(c[1] - LAM) <= 1e-12 * LAM and abs(c[2] - MU2) <= 1e-12 * MU2
    nb, nnz_b = v.n_block_rows, v.nnz_blocks
    assert nb == N and v.block_size == 3 and v.ordered_per_block == 0
    n3, nnz = 3 * nb, 9 * nnz_b
    brows = ctx.to_host(v.rows, nb + 1, np.int64)
    bcols = ctx.to_host(v.columns, nnz_b, np.int32)
    rows = ctx.to_host(ops["scalar_rows"], n3 + 1, np.int64)
    cols = ctx.to_host(ops["scalar_cols"], nnz, np.int32)
    lhs = ctx.to_host(v.values, nnz, np.float64)
    mass = ctx.to_host(ops["mass"], nnz, np.float64)
    cells, coords, _ = mesh.download()
    dyn.close()
    mesh.close()
    # mass total (unit density) = 3 x volume of the jittered box
    xc = coords[cells]
    vol = np.abs(np.linalg.det(np.stack([xc[:, 1] - xc[:, 0], xc[:, 2] - xc[:, 0], xc[:, 3] - xc[:, 0]], 1))).sum() / 6
    del xc
    assert abs(mass.sum() - 3.0 * vol) <= 1e-11 * vol, (mass.sum(), 3 * vol)
    clamped = np.zeros(n3, dtype=bool)
    for d in range(3):
        clamped[3 * fixed + d] = True
    # stiffness part: rigid modes in its kernel on the unclamped rows
    K = lhs - c[0] * mass
    kmax = np.abs(K[np.abs(K) < 1e20]).max()
    X = coords[:N]
    modes = []
    for a in range(3):
        u = np.zeros((N, 3))
        u[:, a] = 1.0
        modes.append(u)
    for w in np.eye(3):
        modes.append(np.cross(w, X))
    Kf = np.where(np.abs(K) < 1e20, K, 0.0)
    worst = 0.0
    for u in modes:
        r = O.spmv(rows, cols, Kf, u.ravel())
        worst = max(worst, np.abs(r[~clamped]).max() / (kmax * np.abs(u).max()))
    del Kf
    assert worst <= 1e-11, worst
    # sampled scalar rows: symmetry, and the clamped rows' penalty diagonal
    rng = np.random.default_rng(128)
    for r in np.concatenate([rng.integers(0, n3, 300), 3 * fixed[:3]]):
        s, e = rows[r], rows[r + 1]
        cc = cols[s:e]
        for t in range(s, e):
            q = int(cols[t])
            tt = rows[q] + np.searchsorted(cols[rows[q]:rows[q + 1]], r)
            assert cols[tt] == r
            if q != r:
                assert abs(lhs[tt] - lhs[t]) <= 1e-13 * kmax
        if clamped[r]:
            assert lhs[s + np.searchsorted(cc, r)] == 1.0e30
    # sampled block rows against the oracle's c0 M + K on the cube neighbourhood
    worst_row = 0.0
    np1 = n + 1
    for g in rng.integers(0, N, 60):
        if g % np1 == 0:
            continue  # clamped node: its rows carry the penalty
        nodes, local, xyz = _kuhn_neighbourhood(n, int(g))
        orp, ocols = O.sparsity(nodes.shape[0], nodes.shape[0], local)
        ov, _ = O.assemble_elasticity_tet(nodes.shape[0], local, xyz, orp, ocols, c[1], c[2], c0=c[0])
        rl = int(np.searchsorted(nodes, g))
        s, e = int(brows[g]), int(brows[g + 1])
        assert np.array_equal(bcols[s:e], nodes[ocols[orp[rl]:orp[rl + 1]]])
        orow = ov[9 * orp[rl]:9 * orp[rl + 1]].reshape(-1, 3, 3)
        grow = lhs[9 * s:9 * e].reshape(3, e - s, 3).transpose(1, 0, 2)  # CSR-row order -> blocks
        worst_row = max(worst_row, np.abs(grow - orow).max() / np.abs(orow).max())
    assert worst_row <= VAL_TOL, worst_row
    print(f"C5 n={n}: {n3} DoF, {nnz_b} blocks; rigid modes of lhs - c0 M: {worst:.2e}; mass total / 3V - 1 = "
          f"{mass.sum() / (3 * vol) - 1:.2e}; sampled block rows vs oracle max rel {worst_row:.2e}")
