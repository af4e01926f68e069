"""Algebraic multigrid preconditioner (afem_solver_opts.amg,
arcanefem_amd/csrc/amg.hip) for the systems the geometric hierarchy does not
cover: Gmsh meshes, caller arrays, refined unstructured meshes.  The PCG with
the aggregation V-cycle reaches the oracle's direct solution (the bar of the
Jacobi-PCG tests), in fewer iterations than point Jacobi, the same bits on every
run, and with penalty rows, eliminated rows and block-3 systems.

The reference's GPU solve is Hypre PCG + BoomerAMG
(femutils/HypreDoFLinearSystem.cc:686-742), external and absent here: only the
solution is compared (parity of the preconditioner itself is unpinned, as for
the reference's own solver)."""
import numpy as np
import pytest

import arcanefem_amd as af
from arcanefem_amd.gmsh import read_gmsh
from oracle import oracle as O

from golden_cases import path

pytestmark = pytest.mark.gpu

SOL_TOL = 1e-10


def _gmsh_mesh(ctx, name):
    gm = read_gmsh(path(name))
    return af.Mesh.from_arrays(ctx, gm.dim, gm.cells, gm.coords), gm


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
    assert st["converged"], (pc, st["iterations"], st["rel_residual"], st["residual_norm"])
    return ls.solution_host().copy(), st


def _dirichlet_nodes(gm, coords, name):
    groups = {"sphere_cut.msh": "horizontal", "L-shape-3D.msh": "bot", "circle_cut.msh": "horizontal"}
    try:
        return gm.group_nodes(groups[name]).astype(np.int32)
    except Exception:  # no such physical group: the lowest layer of nodes
        z = coords[:, coords.shape[1] - 1]
        return np.nonzero(z <= z.min() + 1e-9)[0].astype(np.int32)


@pytest.mark.parametrize("name", ["sphere_cut.msh", "L-shape-3D.msh", "circle_cut.msh"])
def test_amg_poisson_matches_direct(ctx, variant, name):
    """The reference's meshes are small (a few hundred rows): the coarsest
    level is held to 16 rows (AFEM_AMG_DENSE) so that a hierarchy exists."""
    variant("AFEM_AMG_DENSE", "16")
    mesh, gm = _gmsh_mesh(ctx, name)
    cells, coords, _ = mesh.download()
    dn = _dirichlet_nodes(gm, coords, name)
    assert dn.size > 0
    bsr, ls = _poisson(ctx, mesh)
    ls.applyDirichletViaPenalty(dn, 0.5, 1e30)
    x_a, st_a = _solve(ls, "amg")
    ls.applyDirichletViaPenalty(dn, 0.5, 1e30)
    x_j, st_j = _solve(ls, "jacobi")
    orp, ocols = O.sparsity(mesh.n_nodes, mesh.n_own_nodes, cells)
    ovals, orhs = O.assemble_poisson(mesh.n_own_nodes, cells, coords, orp, ocols, 5.5)
    O.dirichlet_penalty(dn, 0.5, 1e30, orp, ocols, ovals, orhs)
    xo = np.linalg.solve(O.csr_to_dense(orp, ocols, ovals), orhs)
    sc = np.abs(xo).max()
    assert np.abs(x_a - xo).max() <= SOL_TOL * sc, np.abs(x_a - xo).max() / sc
    assert np.abs(x_j - xo).max() <= SOL_TOL * sc
    print(f"{name}: {mesh.n_own_nodes} rows, AMG {st_a['iterations']} iterations ({st_a['amg_levels']} levels, "
          f"coarsest {st_a['amg_coarse_rows']}, complexity {st_a['amg_complexity']:.2f}), Jacobi {st_j['iterations']}")
    assert st_a["amg_levels"] >= 2 and 1.0 < st_a["amg_complexity"] < 2.0, st_a
    assert st_j["amg_levels"] == 0
    assert st_a["iterations"] * 2 <= st_j["iterations"], (st_a["iterations"], st_j["iterations"])
    bsr.close()
    mesh.close()


def _refine(cells, coords, levels):
    """Red refinement of tetrahedra (8 children: 4 corners + the inner
    octahedron cut along one diagonal), `levels` times."""
    cells = np.asarray(cells, dtype=np.int64)
    coords = np.asarray(coords, dtype=np.float64)
    for _ in range(levels):
        e = np.concatenate([cells[:, [a, b]] for a, b in ((0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3))])
        e.sort(axis=1)
        uniq, inv = np.unique(e, axis=0, return_inverse=True)
        mid = coords.shape[0] + inv.reshape(6, -1).T
        coords = np.concatenate([coords, 0.5 * (coords[uniq[:, 0]] + coords[uniq[:, 1]])])
        v0, v1, v2, v3 = cells.T
        m01, m02, m03, m12, m13, m23 = mid.T
        cells = np.concatenate([np.stack(c, 1) for c in (
            (v0, m01, m02, m03), (m01, v1, m12, m13), (m02, m12, v2, m23), (m03, m13, m23, v3),
            (m01, m02, m03, m13), (m01, m02, m12, m13), (m02, m03, m13, m23), (m02, m12, m13, m23))])
    return cells.astype(np.int32), coords


def test_amg_refined_unstructured_mesh(ctx):
    """L-shape-3D refined 3x (~80 k nodes): the oracle-free check -- AMG and
    Jacobi reach the same solution at a tight tolerance; AMG in a fraction of
    the iterations; two AMG solves give the same bits."""
    gm = read_gmsh(path("L-shape-3D.msh"))
    cells, coords = _refine(gm.cells, gm.coords, 3)
    mesh = af.Mesh.from_arrays(ctx, 3, cells, coords)
    z = coords[:, 2]
    dn = np.nonzero(z <= z.min() + 1e-9)[0].astype(np.int32)
    bsr, ls = _poisson(ctx, mesh)
    ls.applyDirichletViaPenalty(dn, 0.5, 1e30)
    x_a, st_a = _solve(ls, "amg", rtol=1e-12)
    ls.applyDirichletViaPenalty(dn, 0.5, 1e30)
    x_a2, st_a2 = _solve(ls, "amg", rtol=1e-12)
    ls.applyDirichletViaPenalty(dn, 0.5, 1e30)
    x_j, st_j = _solve(ls, "jacobi", rtol=1e-12)
    print(f"refined L-shape: {mesh.n_own_nodes} rows, AMG {st_a['iterations']} ({st_a['amg_levels']} levels, "
          f"complexity {st_a['amg_complexity']:.2f}, {st_a['solve_ms']:.1f} ms), Jacobi {st_j['iterations']} "
          f"({st_j['solve_ms']:.1f} ms)")
    assert np.array_equal(x_a, x_a2) and st_a["iterations"] == st_a2["iterations"]
    sc = np.abs(x_j).max()
    assert np.abs(x_a - x_j).max() <= 1e-8 * sc, np.abs(x_a - x_j).max() / sc
    assert st_a["iterations"] * 3 <= st_j["iterations"], (st_a["iterations"], st_j["iterations"])
    bsr.close()
    mesh.close()


def test_amg_kcycle(ctx, variant):
    """The K-cycle (two flexible-CG steps on levels 1..k, AFEM_AMG_KCYCLE; 2 by
    default) against the plain V-cycle (0) and the Jacobi-PCG on the refined
    L-shape: the same solution at a tight tolerance, fewer iterations, the
    same bits twice, and the captured graph replays them."""
    gm = read_gmsh(path("L-shape-3D.msh"))
    cells, coords = _refine(gm.cells, gm.coords, 3)
    mesh = af.Mesh.from_arrays(ctx, 3, cells, coords)
    z = coords[:, 2]
    dn = np.nonzero(z <= z.min() + 1e-9)[0].astype(np.int32)
    bsr, ls = _poisson(ctx, mesh)
    ls.applyDirichletViaPenalty(dn, 0.5, 1e30)
    x_j, st_j = _solve(ls, "jacobi", rtol=1e-12)
    xs, its = {}, {}
    for k, g in (("0", "0"), ("2", "0"), ("2", "1"), ("16", "0")):
        variant("AFEM_AMG_KCYCLE", k)
        variant("AFEM_AMG_GRAPH", g)
        ls.applyDirichletViaPenalty(dn, 0.5, 1e30)
        xs[k + g], st = _solve(ls, "amg", rtol=1e-12)
        its[k + g] = st["iterations"]
        assert np.abs(xs[k + g] - x_j).max() <= 1e-8 * np.abs(x_j).max(), (k, g)
    print(f"K-cycle: iterations {its} (Jacobi {st_j['iterations']})")
    assert its["20"] < its["00"] and its["160"] <= its["20"] + 2
    assert np.array_equal(xs["20"], xs["21"]) and its["20"] == its["21"]
    bsr.close()
    mesh.close()


def test_amg_fp32_cycle_products(ctx, variant):
    """The AMG cycle's products on fp32 copies (AFEM_AMG_F32: 0 none, 1 the
    fine level, 2 every level -- the default) and the fused entry / exit
    (AFEM_AMG_FUSE) on the refined L-shape: the PCG's own product stays fp64, so
    every variant reaches the Jacobi-PCG's solution at the tolerance in about the
    same iterations; the fused entry / exit gives the bits of the separate passes."""
    gm = read_gmsh(path("L-shape-3D.msh"))
    cells, coords = _refine(gm.cells, gm.coords, 3)
    mesh = af.Mesh.from_arrays(ctx, 3, cells, coords)
    z = coords[:, 2]
    dn = np.nonzero(z <= z.min() + 1e-9)[0].astype(np.int32)
    bsr, ls = _poisson(ctx, mesh)
    ls.applyDirichletViaPenalty(dn, 0.5, 1e30)
    x_j, _ = _solve(ls, "jacobi", rtol=1e-12)
    xs, its = {}, {}
    for f32, fuse in (("0", "0"), ("1", "1"), ("2", "0"), ("2", "1")):
        variant("AFEM_AMG_F32", f32)
        variant("AFEM_AMG_FUSE", fuse)
        ls.applyDirichletViaPenalty(dn, 0.5, 1e30)
        xs[f32 + fuse], st = _solve(ls, "amg", rtol=1e-12)
        its[f32 + fuse] = st["iterations"]
    print(f"AMG fp32 variants: iterations {its}")
    for k, x in xs.items():
        assert np.abs(x - x_j).max() <= 1e-8 * np.abs(x_j).max(), k
        assert abs(its[k] - its["00"]) <= 3, its
    assert np.array_equal(xs["20"], xs["21"]) and its["20"] == its["21"]
    bsr.close()
    mesh.close()


def test_amg_penalty_beyond_fp32(ctx):
    """A penalty above the fp32 range (1e40) on the clamped rows: the cycle's
    fp32 copies saturate it (never inf, whose product with the constraint rows'
    zero iterate would be NaN), and the AMG-PCG reaches the Jacobi-PCG's solution."""
    gm = read_gmsh(path("L-shape-3D.msh"))
    cells, coords = _refine(gm.cells, gm.coords, 2)
    mesh = af.Mesh.from_arrays(ctx, 3, cells, coords)
    z = coords[:, 2]
    dn = np.nonzero(z <= z.min() + 1e-9)[0].astype(np.int32)
    bsr, ls = _poisson(ctx, mesh)
    ls.applyDirichletViaPenalty(dn, 0.5, 1e40)
    x_j, _ = _solve(ls, "jacobi", rtol=1e-12)
    ls.applyDirichletViaPenalty(dn, 0.5, 1e40)
    x_a, st = _solve(ls, "amg", rtol=1e-12)
    assert np.isfinite(x_a).all()
    assert np.abs(x_a - x_j).max() <= 1e-8 * np.abs(x_j).max()
    assert np.allclose(x_a[dn], 0.5)
    bsr.close()
    mesh.close()


def test_amg_small_system_is_a_direct_solve(ctx):
    """Below 1024 rows the hierarchy is the matrix itself, inverted densely:
    the PCG converges in one or two iterations."""
    mesh, gm = _gmsh_mesh(ctx, "sphere_cut.msh")
    cells, coords, _ = mesh.download()
    dn = _dirichlet_nodes(gm, coords, "sphere_cut.msh")
    bsr, ls = _poisson(ctx, mesh)
    ls.applyDirichletViaPenalty(dn, 0.5, 1e30)
    x_a, st = _solve(ls, "amg")
    assert st["amg_levels"] == 1 and st["iterations"] <= 2, st
    ls.applyDirichletViaPenalty(dn, 0.5, 1e30)
    x_j, _ = _solve(ls, "jacobi")
    assert np.abs(x_a - x_j).max() <= 1e-10 * np.abs(x_j).max()
    bsr.close()
    mesh.close()


def test_amg_row_elimination_and_reuse(ctx, variant):
    """Eliminated rows (identity rows, non-symmetric columns left) stay out of
    the cycle like penalty rows; amg-reuse keeps the hierarchy across solves of
    the same arrays and gives the rebuilt hierarchy's bits."""
    variant("AFEM_AMG_DENSE", "16")
    mesh, gm = _gmsh_mesh(ctx, "sphere_cut.msh")
    cells, coords, _ = mesh.download()
    dn = _dirichlet_nodes(gm, coords, "sphere_cut.msh")
    bsr, ls = _poisson(ctx, mesh)
    ls.applyDirichletViaRowElimination(dn, 0.5)
    x_a, st_a = _solve(ls, "amg")
    ls.applyDirichletViaRowElimination(dn, 0.5)
    x_j, _ = _solve(ls, "jacobi")
    sc = np.abs(x_j).max()
    assert np.abs(x_a - x_j).max() <= 1e-9 * sc
    assert np.abs(x_a[dn] - 0.5).max() <= 1e-12
    ls.applyDirichletViaRowElimination(dn, 0.5)
    x_r1, st_r1 = _solve(ls, "amg-reuse")
    ls.applyDirichletViaRowElimination(dn, 0.5)
    x_r2, st_r2 = _solve(ls, "amg-reuse")
    assert np.array_equal(x_r1, x_r2) and np.array_equal(x_r1, x_a)
    bsr.close()
    mesh.close()


def test_amg_elasticity_block3(ctx, variant):
    """A block-3 elasticity system on a Gmsh mesh (scalar-row aggregation of
    the expanded CSR): the solution of the Jacobi-PCG."""
    variant("AFEM_AMG_DENSE", "32")
    mesh, gm = _gmsh_mesh(ctx, "sphere_cut.msh")
    cells, coords, _ = mesh.download()
    E, NU = 21e5, 0.28
    lam, mu2 = E * NU / ((1 + NU) * (1 - 2 * NU)), E / (1 + NU)
    bsr = af.BSRFormat(mesh, 3).initialize(True)
    bsr.computeSparsity()
    ls = af.DoFLinearSystem().initialize(ctx, 3 * mesh.n_own_nodes, 3 * mesh.n_nodes)
    bsr.assembleElasticityP1Ex(lam, mu2, 0.0, (0.0, 0.0, -1.0), ls.rhsVariable(), rhs_mode="set")
    bsr.toLinearSystem(ls)
    z = coords[:mesh.n_own_nodes, 2]
    fixed = np.nonzero(z <= z.min() + 0.15 * (z.max() - z.min()))[0]  # a clamped bottom slab
    dofs = (3 * fixed[:, None] + np.arange(3)[None, :]).ravel().astype(np.int32)
    ls.applyDirichletViaPenalty(dofs, 0.0, 1e30)
    x_a, st_a = _solve(ls, "amg", rtol=1e-12)
    ls.applyDirichletViaPenalty(dofs, 0.0, 1e30)
    x_j, st_j = _solve(ls, "jacobi", rtol=1e-12)
    print(f"sphere elasticity: AMG {st_a['iterations']}, Jacobi {st_j['iterations']}")
    sc = np.abs(x_j).max()
    assert np.abs(x_a - x_j).max() <= 1e-7 * sc, np.abs(x_a - x_j).max() / sc
    assert st_a["iterations"] < st_j["iterations"]
    bsr.close()
    mesh.close()


def test_amg_option_validation(ctx):
    mesh = af.Mesh.structured(ctx, 3, 4)
    ls = af.DoFLinearSystem().initialize(ctx, 3 * mesh.n_own_nodes)
    o = af._capi.SolverOpts()
    af._capi.call("afem_ls_get_solver_options", ls.impl, af._capi.ctypes.byref(o))
    o.amg = 3
    with pytest.raises(af.AfemError):
        af._capi.call("afem_ls_set_solver_options", ls.impl, af._capi.ctypes.byref(o))
    o.amg, o.precond_block = 1, 3
    with pytest.raises(af.AfemError):
        af._capi.call("afem_ls_set_solver_options", ls.impl, af._capi.ctypes.byref(o))
    mesh.close()


def test_amg_graph_replay_bitwise(ctx, variant):
    """AFEM_AMG_GRAPH=1 (the V-cycle captured once per solve and replayed as a
    HIP graph) runs the same kernels in the same order: the same bits."""
    variant("AFEM_AMG_DENSE", "16")
    mesh, gm = _gmsh_mesh(ctx, "sphere_cut.msh")
    cells, coords, _ = mesh.download()
    dn = _dirichlet_nodes(gm, coords, "sphere_cut.msh")
    bsr, ls = _poisson(ctx, mesh)
    xs = {}
    for g in ("0", "1"):
        variant("AFEM_AMG_GRAPH", g)
        ls.applyDirichletViaPenalty(dn, 0.5, 1e30)
        xs[g], st = _solve(ls, "amg")
        assert st["amg_levels"] >= 2
    assert np.array_equal(xs["0"], xs["1"])
    bsr.close()
    mesh.close()


def test_amg_reuse_rebuilds_on_new_values(ctx, variant):
    """amg-reuse keeps the hierarchy only while the CSR arrays and sizes are
    the same: a second setCSRValues with the same sizes (new device
    buffers that may sit at the old addresses) rebuilds it, and the solve of the
    doubled matrix is half the first solution."""
    variant("AFEM_AMG_DENSE", "16")
    mesh, gm = _gmsh_mesh(ctx, "sphere_cut.msh")
    cells, coords, _ = mesh.download()
    dn = _dirichlet_nodes(gm, coords, "sphere_cut.msh")
    bsr, ls0 = _poisson(ctx, mesh)
    rows, cols, vals = bsr.download()
    rhs = ls0.rhs_host()
    n = mesh.n_own_nodes
    ls = af.DoFLinearSystem().initialize(ctx, n, mesh.n_nodes)
    sols = []
    for scale in (1.0, 2.0):
        v = vals * scale
        ls.setCSRValues(rows[:-1], None, cols, v)
        ctx.to_device(ls.rhsVariable(), rhs)
        ls.applyDirichletViaPenalty(dn, 0.5, 1e30)
        x, st = _solve(ls, "amg-reuse")
        assert st["amg_setup_ms"] > 0.0, (scale, st)  # built (first) / rebuilt (new values)
        ctx.to_device(ls.rhsVariable(), rhs)
        ls.applyDirichletViaPenalty(dn, 0.5, 1e30)
        x2, st2 = _solve(ls, "amg-reuse")
        assert st2["amg_setup_ms"] == 0.0 and np.array_equal(x, x2)  # kept
        sols.append(x)
    free = np.ones(n, dtype=bool)
    free[dn] = False
    # 2 A x' = b on the free rows with the same Dirichlet values: x' - g = (x - g) / 2
    g = 0.5
    assert np.abs((sols[1][free] - g) - 0.5 * (sols[0][free] - g)).max() <= 1e-9 * np.abs(sols[0]).max()
    ls.reset()
    ls0.reset()
    bsr.close()
    mesh.close()


def test_amg_reuse_and_time_step_change(ctx, variant):
    """Elastodynamics with the amg-reuse preconditioner: a dt change (passmo's
    shortened last step, afem_elastodynamics_set_time_step) changes c0 M + K, so
    the hierarchy is rebuilt at the next step; states equal the
    Jacobi-PCG run's."""
    from arcanefem_amd.elastodynamics import Elastodynamics3D

    variant("AFEM_AMG_DENSE", "32")
    mesh = af.Mesh.structured(ctx, 3, 6)
    cells, coords, _ = mesh.download()
    fixed = np.nonzero(coords[:, 0] < 0.5 / 6)[0]
    kw = dict(body_force=(0.0, -9.81, 1.0), fixed_nodes=fixed, rtol=1e-13)
    runs = {}
    for pc in ("amg-reuse", "jacobi"):
        sim = Elastodynamics3D(ctx, mesh, 21e5, 0.28, 1.0, 1e-3, preconditioner=pc, **kw)
        setups = []
        for k in range(5):
            if k == 3:
                sim.setTimeStep(4e-4)
            st = sim.step()
            assert st["converged"], (pc, k, st)
            setups.append(st["amg_setup_ms"])
        if pc == "amg-reuse":
            assert setups[0] > 0 and setups[1] == 0 and setups[2] == 0, setups
            assert setups[3] > 0 and setups[4] == 0, setups  # rebuilt after the dt change, then kept
        runs[pc] = sim.state_host()
        sim.close()
    for a, b in zip(runs["amg-reuse"], runs["jacobi"]):
        assert np.abs(a - b).max() <= 1e-8 * np.abs(b).max()
    mesh.close()
