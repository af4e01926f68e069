"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle.

Tolerances (BASELINE.json north_star: "assembled CSR and solution vector
matching the CPU reference to 1e-10 relative"):
  * structure (row offsets, columns): bit-exact;
  * CSR values and RHS: |gpu - oracle| <= 1e-12 * max|oracle| per entry
    (only the summation order and the element-formula evaluation order
    differ: ~1e-16 relative per entry);
  * solution: <= 1e-10 relative (max-norm) against a direct dense solve of
    the oracle system on small meshes; the reference goldens at their own
    1e-4 gate (checkNodeResultFile) and at the restatement's measured error.
"""
import numpy as np
import pytest

import arcanefem_amd as af
from arcanefem_amd.gmsh import read_gmsh, read_node_result_file
from oracle import oracle as O

from golden_cases import CASES, GOLDEN_TOL, path

pytestmark = pytest.mark.gpu

VAL_TOL = 1e-12
SOL_TOL = 1e-10


CUBES_V = 16 | 32 | 64 | 256 | 512 | 1024  # cubes.hip kCubesV


def _assemble_gpu(ctx, mesh, f):
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    bsr.computeSparsity()
    ls = af.DoFLinearSystem().initialize(ctx, mesh.n_own_nodes, mesh.n_nodes)
    bsr.assemblePoissonP1(1.0, 0.0 if f is None else f, ls.rhsVariable())
    bsr.toLinearSystem(ls)
    return bsr, ls


def _check_values(vals, ovals):
    scale = np.abs(ovals).max()
    err = np.abs(vals - ovals).max() / scale
    assert err <= VAL_TOL, f"CSR values differ from the oracle: {err:.3e}"
    return err


# ---------------------------------------------------------------- mesh generator
@pytest.mark.parametrize("dim,n,nz,nranks", [(3, 5, 7, 1), (3, 4, 9, 3), (2, 9, None, 1), (2, 6, None, 4)])
def test_structured_generator_matches_spec(ctx, dim, n, nz, nranks):
    for rank in range(nranks):
        m = af.Mesh.structured(ctx, dim, n, nz=nz, jitter=0.2, seed=7, nranks=nranks, rank=rank)
        cells, coords, l2g = m.download()
        ref = O.structured_mesh(dim, n, nz=nz, jitter=0.2, seed=7, nranks=nranks, rank=rank)
        assert m.n_own_nodes == ref["n_own"] and m.n_nodes == ref["n_local"]
        assert np.array_equal(cells, ref["cells"])
        assert np.array_equal(l2g, ref["local_to_global"])
        assert np.array_equal(coords, ref["coords"]), "generator coordinates are not bitwise equal to the spec"
        assert np.array_equal(m.bottom_nodes(), ref["dirichlet"])
        m.close()


# ---------------------------------------------------------------- assembly parity
@pytest.mark.parametrize("dim,n", [(3, 1), (3, 2), (3, 11), (2, 1), (2, 17)])
def test_structured_assembly_parity(ctx, dim, n):
    mesh = af.Mesh.structured(ctx, dim, n)
    bsr, ls = _assemble_gpu(ctx, mesh, 5.5)
    rows, cols, vals = bsr.download()
    cells, coords, _ = mesh.download()
    orp, ocols = O.sparsity(mesh.n_nodes, mesh.n_own_nodes, cells)
    ovals, orhs = O.assemble_poisson(mesh.n_own_nodes, cells, coords, orp, ocols, 5.5)
    assert np.array_equal(rows, orp)
    assert np.array_equal(cols, ocols)
    _check_values(vals, ovals)
    rhs = ls.rhs_host()
    assert np.abs(rhs - orhs).max() <= VAL_TOL * np.abs(orhs).max()


def test_boundary_aware_order_on_thin_boxes(ctx):
    """The boundary-aware brick order (interior bricks, face tiles, edge runs,
    corners) on boxes one to a few cells thick along an axis (empty interiors,
    faces that coincide, edges without interior nodes): every owned node in
    exactly one slice (checked by the structure build) and the oracle's
    matrix."""
    for n, nz in [(1, 1), (1, 4), (3, 1), (4, 2), (9, 3), (2, 7), (33, 2)]:
        mesh = af.Mesh.structured(ctx, 3, n, nz)
        bsr, ls = _assemble_gpu(ctx, mesh, 5.5)
        assert bsr.stats()["brick_order"] == 1
        rows, cols, vals = bsr.download()
        cells, coords, _ = mesh.download()
        orp, ocols = O.sparsity(mesh.n_nodes, mesh.n_own_nodes, cells)
        ovals, orhs = O.assemble_poisson(mesh.n_own_nodes, cells, coords, orp, ocols, 5.5)
        assert np.array_equal(rows, orp) and np.array_equal(cols, ocols), (n, nz)
        _check_values(vals, ovals)
        assert np.abs(ls.rhs_host() - orhs).max() <= VAL_TOL * np.abs(orhs).max(), (n, nz)


@pytest.mark.parametrize("case", list(CASES))
def test_golden_mesh_assembly_parity(ctx, case):
    mfile, f, bcs, gfile, P = CASES[case]
    gm = read_gmsh(path(mfile))
    mesh = af.Mesh.from_arrays(ctx, gm.dim, gm.cells, gm.coords)
    bsr, ls = _assemble_gpu(ctx, mesh, f)
    rows, cols, vals = bsr.download()
    orp, ocols = O.sparsity(gm.n_nodes, gm.n_nodes, gm.cells)
    ovals, orhs = O.assemble_poisson(gm.n_nodes, gm.cells, gm.coords, orp, ocols, 0.0 if f is None else f)
    assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
    _check_values(vals, ovals)
    assert np.abs(ls.rhs_host() - orhs).max() <= VAL_TOL * max(np.abs(orhs).max(), 1e-300)


def test_assembly_bitwise_reproducible(ctx):
    mesh = af.Mesh.structured(ctx, 3, 14, seed=3)
    bsr, ls = _assemble_gpu(ctx, mesh, 2.0)
    _, _, v1 = bsr.download()
    r1 = ls.rhs_host()
    for _ in range(2):
        bsr.assemblePoissonP1(1.0, 2.0, ls.rhsVariable(), rhs_mode="set")
        _, _, v2 = bsr.download()
        assert np.array_equal(v1, v2)
        assert np.array_equal(r1, ls.rhs_host())


@pytest.mark.parametrize("n,nz,zs", [(1, 1, None), (2, 5, None), (6, 6, None), (7, 3, 2), (8, 9, 1), (13, 20, 3),
                                     (20, 7, None)])
def test_cube_kernel_matches_oracle(ctx, variant, n, nz, zs):
    """The cell-first cube kernel (cubes.hip, the default on generator boxes):
    boxes whose line lengths are and are not multiples of the 7-row columns,
    thin boxes, and z segments of 1-3 layers (AFEM_CUBES_ZS): values and RHS
    against the oracle (1e-12 per entry) and against the row-strip kernels
    (AFEM_ASSEMBLY_CUBES=0, the same to rounding); RHS added and set; and
    bitwise run-to-run."""
    variant("AFEM_ASSEMBLY_CUBES", "1")  # opt-in
    if zs is not None:
        variant("AFEM_CUBES_ZS", str(zs))
    mesh = af.Mesh.structured(ctx, 3, n, nz, jitter=0.2, seed=31)
    bsr, ls = _assemble_gpu(ctx, mesh, 5.5)
    assert bsr.stats()["last_kernel"] == 10  # AFEM_KERNEL_CUBES
    rows, cols, vals = bsr.download()
    rhs = ls.rhs_host()
    cells, coords, _ = mesh.download()
    orp, ocols = O.sparsity(mesh.n_nodes, mesh.n_own_nodes, cells)
    ovals, orhs = O.assemble_poisson(mesh.n_own_nodes, cells, coords, orp, ocols, 5.5)
    assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
    _check_values(vals, ovals)
    assert np.abs(rhs - orhs).max() <= VAL_TOL * np.abs(orhs).max()
    # RHS add mode on top, and the set mode again: reproducible bits
    bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable(), rhs_mode="add")
    assert np.array_equal(ls.rhs_host(), rhs + rhs)
    bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable(), rhs_mode="set")
    assert np.array_equal(bsr.download()[2], vals) and np.array_equal(ls.rhs_host(), rhs)
    variant("AFEM_ASSEMBLY_CUBES", "0")
    bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable(), rhs_mode="set")
    assert bsr.stats()["last_kernel"] != 10
    v_strip = bsr.download()[2]
    assert np.abs(vals - v_strip).max() <= VAL_TOL * np.abs(v_strip).max()
    assert np.abs(ls.rhs_host() - rhs).max() <= VAL_TOL * np.abs(rhs).max()


@pytest.mark.parametrize("nranks,stride,carry,nz,zs", [(2, "64", "1", 11, None), (3, "64", "1", 11, None),
                                                     (3, "49", "0", 11, None), (2, "64", "0", 11, None),
                                                     (2, "64", "1", 11, "1"), (3, "64", "1", 11, "2"),
                                                     (4, "64", "1", 5, "2"), (3, "64", "1", 2, None),
                                                     (5, "64", "1", 6, "1")])
def test_cube_kernel_on_slabs(ctx, variant, nranks, stride, carry, nz, zs):
    """z-slab subdomains (owned layers, then the ghost layer below, then the one
    above: a row next to the ghost layer below has its -z columns LAST in id
    order): every slab's matrix and RHS against the oracle on the same
    subdomain, through the cube kernel.  z segments of 1 and 2 layers
    (AFEM_CUBES_ZS) start inside a slab next to its ghost layers,
    and nz = 2 on 3 ranks / 6 on 5 leave slabs of ONE owned node layer."""
    variant("AFEM_ASSEMBLY_CUBES", "1")  # opt-in
    variant("AFEM_CUBES_STRIDE", stride)  # accumulator planes of 64 (default) or 49 rows
    variant("AFEM_CUBES_CARRY", carry)  # top-face sums carried in registers (default) or not
    variant("AFEM_CUBES_ZS", zs)
    owned = []
    for rank in range(nranks):
        mesh = af.Mesh.structured(ctx, 3, 9, nz=nz, jitter=0.2, seed=13, nranks=nranks, rank=rank)
        owned.append(mesh.n_own_nodes // 100)
        bsr, ls = _assemble_gpu(ctx, mesh, 2.5)
        assert bsr.stats()["last_kernel"] == 10
        rows, cols, vals = bsr.download()
        cells, coords, _ = mesh.download()
        orp, ocols = O.sparsity(mesh.n_nodes, mesh.n_own_nodes, cells)
        ovals, orhs = O.assemble_poisson(mesh.n_own_nodes, cells, coords, orp, ocols, 2.5)
        assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
        _check_values(vals, ovals)
        assert np.abs(ls.rhs_host() - orhs).max() <= VAL_TOL * np.abs(orhs).max()
        mesh.close()
    assert sum(owned) == nz + 1
    if nz in (2, 6):
        assert min(owned) == 1


def test_uniform_strip_variant(ctx, variant):
    variant("AFEM_ASSEMBLY_CUBES", "0")  # the row-strip family (generator boxes default to cubes.hip)
    # interior 4x4x4 bricks of a structured box share one strip topology and
    # run the uniform-control kernel; it must give the general kernel's bits
    # and match the oracle
    mesh = af.Mesh.structured(ctx, 3, 23, seed=11)
    bsr, ls = _assemble_gpu(ctx, mesh, 5.5)
    st = bsr.stats()
    # (boundary-aware order: faces, box edges and corners in their own slices,
    # so at this size every slice is uniform)
    assert st["brick_order"] == 1 and 0 < st["uniform_slices"] <= st["n_slices"]
    _, _, v_uni = bsr.download()
    r_uni = ls.rhs_host()
    variant("AFEM_ASSEMBLY_UNIFORM", "0")
    bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable(), rhs_mode="set")
    rows, cols, v_gen = bsr.download()
    assert np.array_equal(v_uni, v_gen), "uniform and general strip kernels differ"
    assert np.array_equal(r_uni, ls.rhs_host())
    cells, coords, _ = mesh.download()
    orp, ocols = O.sparsity(mesh.n_nodes, mesh.n_own_nodes, cells)
    ovals, orhs = O.assemble_poisson(mesh.n_own_nodes, cells, coords, orp, ocols, 5.5)
    assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
    _check_values(v_uni, ovals)
    assert np.abs(r_uni - orhs).max() <= VAL_TOL * np.abs(orhs).max()


@pytest.mark.parametrize("n", [23, 40])
def test_stencil_instance_bitwise(ctx, variant, n):
    """Interior bricks of a Kuhn box match the compiled-in strip signature
    (stencil_sigs.inc) and run k_assemble_stencil (register accumulators): the
    same bits as the uniform instance (AFEM_ASSEMBLY_STENCIL=0) and the general
    instance (AFEM_ASSEMBLY_UNIFORM=0), and the oracle's values."""
    variant("AFEM_ASSEMBLY_CUBES", "0")  # the row-strip family (generator boxes default to cubes.hip)
    mesh = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=7)
    bsr, ls = _assemble_gpu(ctx, mesh, 5.5)
    st = bsr.stats()
    print("slices", st["n_slices"], "uniform", st["uniform_slices"], "stencil", st["stencil_slices"])
    assert st["stencil_sig"] == 0 and 0 < st["stencil_slices"] <= st["uniform_slices"]
    _, _, v_k = bsr.download()
    r_k = ls.rhs_host()
    variant("AFEM_ASSEMBLY_STENCIL", "0")
    bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable(), rhs_mode="set")
    _, _, v_uni = bsr.download()
    assert np.array_equal(v_k, v_uni), f"stencil and uniform instances differ in {np.count_nonzero(v_k != v_uni)} values"
    assert np.array_equal(r_k, ls.rhs_host())
    variant("AFEM_ASSEMBLY_UNIFORM", "0")
    bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable(), rhs_mode="set")
    rows, cols, v_gen = bsr.download()
    assert np.array_equal(v_k, v_gen)
    assert np.array_equal(r_k, ls.rhs_host())
    cells, coords, _ = mesh.download()
    orp, ocols = O.sparsity(mesh.n_nodes, mesh.n_own_nodes, cells)
    ovals, orhs = O.assemble_poisson(mesh.n_own_nodes, cells, coords, orp, ocols, 5.5)
    assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
    _check_values(v_k, ovals)
    assert np.abs(r_k - orhs).max() <= VAL_TOL * np.abs(orhs).max()


def test_edge_slices_folded_into_general_list(ctx, variant):
    """Box edges and corners (boundary-aware order: runs of 64 along the 12
    edges, one slice per corner) are uniform slices without a compiled-in
    signature; beside enough stencil slices they join the compact general list
    (one launch before the stencil kernel).  Same bits as keeping them on the
    uniform instance (AFEM_ASSEMBLY_FOLD=0) and as the general instance."""
    variant("AFEM_ASSEMBLY_CUBES", "0")  # the row-strip family (generator boxes default to cubes.hip)
    mesh = af.Mesh.structured(ctx, 3, 100, jitter=0.2, seed=5)
    bsr, ls = _assemble_gpu(ctx, mesh, 3.0)
    st = bsr.stats()
    assert st["stencil_slices"] < st["uniform_slices"] <= st["n_slices"]
    assert st["uniform_instance_slices"] == 0 and st["general_slices"] > 0, st
    _, _, v_fold = bsr.download()
    r_fold = ls.rhs_host()
    variant("AFEM_ASSEMBLY_FOLD", "0")
    bsr2, ls2 = _assemble_gpu(ctx, mesh, 3.0)
    st2 = bsr2.stats()
    assert st2["uniform_instance_slices"] == st["uniform_slices"] - st["stencil_slices"], st2
    _, _, v_nf = bsr2.download()
    assert np.array_equal(v_fold, v_nf) and np.array_equal(r_fold, ls2.rhs_host())
    variant("AFEM_ASSEMBLY_UNIFORM", "0")
    bsr2.assemblePoissonP1(1.0, 3.0, ls2.rhsVariable(), rhs_mode="set")
    _, _, v_gen = bsr2.download()
    assert np.array_equal(v_fold, v_gen) and np.array_equal(r_fold, ls2.rhs_host())


def test_isolated_node_and_ragged_rows(ctx):
    # two tets sharing a face + one node touched by no cell (empty row apart
    # from the diagonal the reference always inserts, BSRFormat.h:679)
    coords = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1], [1, 1, 1], [5, 5, 5]], dtype=np.float64)
    cells = np.array([[0, 1, 2, 3], [1, 2, 3, 4]], dtype=np.int32)
    mesh = af.Mesh.from_arrays(ctx, 3, cells, coords)
    bsr, ls = _assemble_gpu(ctx, mesh, 1.0)
    rows, cols, vals = bsr.download()
    orp, ocols = O.sparsity(6, 6, cells)
    ovals, orhs = O.assemble_poisson(6, cells, coords, orp, ocols, 1.0)
    assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
    assert rows[6] - rows[5] == 1 and cols[rows[5]] == 5
    _check_values(vals, ovals)


def test_ghost_rows_are_not_materialised(ctx):
    # slab 1 of 3: rows = owned nodes only, ghost columns >= n_own (isOwn filter, BSRFormat.h:815)
    mesh = af.Mesh.structured(ctx, 3, 6, nz=8, nranks=3, rank=1)
    bsr, ls = _assemble_gpu(ctx, mesh, 5.5)
    rows, cols, vals = bsr.download()
    cells, coords, _ = mesh.download()
    orp, ocols = O.sparsity(mesh.n_nodes, mesh.n_own_nodes, cells)
    ovals, orhs = O.assemble_poisson(mesh.n_own_nodes, cells, coords, orp, ocols, 5.5)
    assert rows.shape[0] == mesh.n_own_nodes + 1
    assert cols.max() >= mesh.n_own_nodes
    assert np.array_equal(cols, ocols)
    _check_values(vals, ovals)
    assert np.abs(ls.rhs_host() - orhs).max() <= VAL_TOL * np.abs(orhs).max()


@pytest.mark.parametrize("dim,n,nz,nranks,rank", [(3, 9, 13, 3, 1), (3, 7, 10, 2, 0), (2, 21, None, 2, 1),
                                                   (2, 30, None, 3, 2)])
def test_slab_assembly_parity(ctx, dim, n, nz, nranks, rank):
    # brick-ordered slices over slabs whose owned layer count is not a
    # multiple of the brick height (partial bricks, idle lanes)
    mesh = af.Mesh.structured(ctx, dim, n, nz=nz, nranks=nranks, rank=rank)
    bsr, ls = _assemble_gpu(ctx, mesh, 3.0)
    st = bsr.stats()
    assert st["brick_order"] == 1 and st["rows_per_block"] == 64
    rows, cols, vals = bsr.download()
    cells, coords, _ = mesh.download()
    orp, ocols = O.sparsity(mesh.n_nodes, mesh.n_own_nodes, cells)
    ovals, orhs = O.assemble_poisson(mesh.n_own_nodes, cells, coords, orp, ocols, 3.0)
    assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
    _check_values(vals, ovals)
    assert np.abs(ls.rhs_host() - orhs).max() <= VAL_TOL * np.abs(orhs).max()


def _elasticity_meshes(ctx, which):
    if which == "bar":
        gm = read_gmsh(path("bar.msh"))
        return af.Mesh.from_arrays(ctx, 2, gm.cells, gm.coords)
    if which == "box":
        return af.Mesh.structured(ctx, 2, 37)
    return af.Mesh.structured(ctx, 2, 19, nranks=3, rank=1)


@pytest.mark.parametrize("which", ["bar", "box", "slab"])
@pytest.mark.parametrize("use_csr", [False, True])
def test_elasticity_assembly_parity(ctx, which, use_csr):
    # block-2 P1 elasticity (modules/elasticity/FemModule.h:112-140) in both
    # value layouts of BSRFormat: per block and per scalar row (Hypre CSR)
    mesh = _elasticity_meshes(ctx, which)
    lam, mu2 = 1.2e5, 2 * 8.1e4
    bsr = af.BSRFormat(mesh, 2).initialize(use_csr)
    bsr.computeSparsity()
    bsr.assembleElasticityP1(lam, mu2)
    rows, cols, vals = bsr.download()
    cells, coords, _ = mesh.download()
    orp, ocols = O.sparsity(mesh.n_nodes, mesh.n_own_nodes, cells)
    ovals = O.assemble_elasticity_tri(mesh.n_own_nodes, cells, coords, orp, ocols, lam, mu2)
    if use_csr:
        ovals = O.blocks_to_row_order(orp, ovals)
    assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
    _check_values(vals, ovals)


def test_row_sums_vanish_at_scale(ctx):
    # size-independent property on a ~1.1M DoF mesh: constants are in the
    # kernel of the Laplacian (rows sum to 0 up to rounding) and K is symmetric
    mesh = af.Mesh.structured(ctx, 3, 103)
    bsr, ls = _assemble_gpu(ctx, mesh, 5.5)
    rows, cols, vals = bsr.download()
    rid = np.repeat(np.arange(rows.shape[0] - 1), np.diff(rows))
    sums = np.bincount(rid, weights=vals)
    diag = vals[cols == rid]
    assert np.abs(sums).max() <= 1e-12 * diag.max()
    # symmetry: a_ij == a_ji (bitwise up to the summation order)
    key = rid.astype(np.int64) * (rows.shape[0]) + cols
    keyT = cols.astype(np.int64) * (rows.shape[0]) + rid
    order = np.argsort(key)
    posT = np.searchsorted(key[order], keyT)
    assert np.abs(vals - vals[order][posT]).max() <= 1e-14 * diag.max()
    # RHS sums to f * volume of the box (jitter moves boundary nodes: compare
    # with the sum of cell volumes the oracle's element routine returns on a sample)
    rhs = ls.rhs_host()
    assert abs(rhs.sum() - 5.5) < 0.05 * 5.5


# ---------------------------------------------------------------- BC + solve parity
def _oracle_system(gm_cells, coords, n_own, n_nodes, f, bcs, P):
    orp, ocols = O.sparsity(n_nodes, n_own, gm_cells)
    ovals, orhs = O.assemble_poisson(n_own, gm_cells, coords, orp, ocols, 0.0 if f is None else f)
    for ids, g in bcs:
        O.dirichlet_penalty(ids, g, P, orp, ocols, ovals, orhs)
    return orp, ocols, ovals, orhs


@pytest.mark.parametrize("case", list(CASES))
@pytest.mark.parametrize("method", ["auto", "pcg"])
def test_golden_solve(ctx, case, method):
    mfile, f, bcs, gfile, P = CASES[case]
    gm = read_gmsh(path(mfile))
    mesh = af.Mesh.from_arrays(ctx, gm.dim, gm.cells, gm.coords)
    bsr, ls = _assemble_gpu(ctx, mesh, f)
    groups = [(gm.group_nodes(g), v) for g, v in bcs]
    for ids, v in groups:
        ls.applyDirichletViaPenalty(ids, v, P)
    ls.setSolverOptions(rtol=1e-14, max_iter=20000, method=method)
    st = ls.solve()
    assert st["converged"], st
    x = ls.solution_host()
    # against the oracle's direct solve of the same system
    orp, ocols, ovals, orhs = _oracle_system(gm.cells, gm.coords, gm.n_nodes, gm.n_nodes, f, groups, P)
    xo = np.linalg.solve(O.csr_to_dense(orp, ocols, ovals), orhs)
    assert np.abs(x - xo).max() / np.abs(xo).max() <= SOL_TOL
    # the matrix after BCs equals the oracle's
    _, _, vals = bsr.download()
    _check_values(vals, ovals)
    # against the reference golden file
    gold = read_node_result_file(path(gfile))
    nerr, mx = O.check_node_result({int(t): x[i] for i, t in enumerate(gm.node_tags)}, gold, 1e-4)
    assert nerr == 0
    assert mx <= GOLDEN_TOL[case] * 1.5


@pytest.mark.parametrize("dim,n", [(3, 12), (2, 40)])
def test_structured_solve_parity(ctx, dim, n):
    mesh = af.Mesh.structured(ctx, dim, n)
    bsr, ls = _assemble_gpu(ctx, mesh, 5.5)
    bottom = mesh.bottom_nodes()
    ls.applyDirichletViaPenalty(bottom, 0.5, 1e30)
    ls.setSolverOptions(rtol=1e-14, max_iter=20000)
    st = ls.solve()
    assert st["converged"]
    x = ls.solution_host()
    cells, coords, _ = mesh.download()
    orp, ocols, ovals, orhs = _oracle_system(cells, coords, mesh.n_own_nodes, mesh.n_nodes, 5.5, [(bottom, 0.5)],
                                             1e30)
    A = O.csr_to_dense(orp, ocols, ovals)
    xo = np.linalg.solve(A, orhs)
    assert np.abs(x - xo).max() / np.abs(xo).max() <= SOL_TOL
    # and against the oracle's own Jacobi-PCG
    xp, it, res, _ = O.pcg_jacobi(orp, ocols, ovals, orhs, rtol=1e-14, max_iter=20000)
    assert np.abs(x - xp).max() / np.abs(xp).max() <= SOL_TOL


# ---------------------------------------------------------------- other plugin paths
def test_matrix_add_value_path_matches_csr_path(ctx):
    """CPU-module semantics (_assembleBilinear with matrixAddValue per entry,
    modules/poisson/FemModule.cc:300-323; Aleph/Sequential add+set) on the GPU
    solver: same solution as the BSR path."""
    gm = read_gmsh(path("L-shape.msh"))
    ls = af.DoFLinearSystem().initialize(ctx, gm.n_nodes)
    rhs = np.zeros(gm.n_nodes)
    for c in gm.cells:
        K, area = O.element_tri3(gm.coords[c])
        for a in range(3):
            for b in range(3):
                ls.matrixAddValue(int(c[a]), int(c[b]), float(K[a, b]))
            rhs[c[a]] += -5.5 * area / 3
    for d in gm.group_nodes("boundary"):
        ls.matrixSetValue(int(d), int(d), 1e30)
        rhs[d] = 1e30 * 0.5
    ls.set_rhs_host(rhs)
    ls.setSolverOptions(rtol=1e-14, max_iter=20000)
    st = ls.solve()
    assert st["converged"]
    x = ls.solution_host()
    gold = read_node_result_file(path("poisson_test_ref_L-shape_2D.txt"))
    nerr, mx = O.check_node_result({int(t): x[i] for i, t in enumerate(gm.node_tags)}, gold, 1e-4)
    assert nerr == 0 and mx < 1e-10


def test_set_csr_values_host_view_and_row_elimination(ctx):
    gm = read_gmsh(path("circle_cut.msh"))
    orp, ocols = O.sparsity(gm.n_nodes, gm.n_nodes, gm.cells)
    ovals, orhs = O.assemble_poisson(gm.n_nodes, gm.cells, gm.coords, orp, ocols, 5.5)
    ls = af.DoFLinearSystem().initialize(ctx, gm.n_nodes)
    ls.setCSRValues(orp[:-1].astype(np.int32), np.diff(orp).astype(np.int32), ocols, ovals)
    assert ls.hasSetCSRValues()
    ls.set_rhs_host(orhs)
    ids = gm.group_nodes("horizontal")
    ls.applyDirichletViaRowElimination(ids, 0.5)
    ls.setSolverOptions(rtol=1e-14)
    st = ls.solve()
    assert st["converged"]
    x = ls.solution_host()
    v2 = ovals.copy()
    r2 = orhs.copy()
    O.row_elimination(ids, 0.5, orp, ocols, v2, r2)
    xo = np.linalg.solve(O.csr_to_dense(orp, ocols, v2), r2)
    assert np.abs(x - xo).max() / np.abs(xo).max() <= SOL_TOL
    assert np.allclose(x[ids], 0.5, rtol=0, atol=1e-13)


def test_errors_are_raised_not_swallowed(ctx):
    mesh = af.Mesh.structured(ctx, 2, 3)
    bsr, ls = _assemble_gpu(ctx, mesh, 1.0)
    with pytest.raises(af.AfemError) as e:
        bsr.setValue(0, mesh.n_own_nodes - 1, 1.0)  # far corner: not a neighbour of node 0
    assert e.value.code == 5
    with pytest.raises(af.AfemError):
        ls.matrixAddValue(0, mesh.n_own_nodes - 1, 1.0)
    with pytest.raises(af.AfemError):
        af.BSRFormat(mesh, 4).initialize()
    b2 = af.BSRFormat(mesh, 1).initialize()
    with pytest.raises(af.AfemError) as e:
        b2.assemblePoissonP1(1.0, 0.0, None)  # before computeSparsity
    assert e.value.code == 4


def test_spmv_matches_oracle(ctx):
    mesh = af.Mesh.structured(ctx, 3, 9)
    bsr, ls = _assemble_gpu(ctx, mesh, 1.0)
    rows, cols, vals = bsr.download()
    x = np.random.default_rng(0).standard_normal(mesh.n_nodes)
    dx = ctx.malloc(x.nbytes)
    dy = ctx.malloc(8 * mesh.n_own_nodes)
    ctx.to_device(dx, x)
    ls.spmv(dx, dy)
    y = ctx.to_host(dy, mesh.n_own_nodes, np.float64)
    yo = O.spmv(rows, cols, vals, x)
    assert np.abs(y - yo).max() <= 1e-13 * np.abs(yo).max()
    ctx.free(dx)
    ctx.free(dy)


@pytest.mark.parametrize("dim,n", [(3, 12), (2, 40)])
@pytest.mark.parametrize("order", ["default", "hilbert", "morton", "node"])
def test_random_node_permutation(ctx, variant, dim, n, order):
    # SURVEY §8d robustness variant: the structured mesh with a seeded random
    # node and cell numbering, handed over as arrays.  Default: a 3D mesh whose
    # owned nodes sit on a lattice gets the brick order of that lattice
    # (recovered from the coordinates, brick_order 2; in the generator's
    # numbering its bricks reach the uniform / stencil instances,
    # test_lattice_order_matches_generator_box); other meshes (2D here) follow a
    # Hilbert curve of the node coordinates.  AFEM_ORDER=hilbert / morton /
    # node force the Hilbert curve, a Morton curve or the caller's node order
    # (read at every computeSparsity).  The assembled matrix must be the
    # permuted matrix of the unpermuted box in every case.
    ref = O.structured_mesh(dim, n, jitter=0.2, seed=20250220)
    rng = np.random.default_rng(1234)
    nn = ref["n_local"]
    p = rng.permutation(nn)              # new id of old node i is p[i]
    cells = p[ref["cells"]].astype(np.int32)[rng.permutation(ref["cells"].shape[0])]
    coords = np.empty_like(ref["coords"])
    coords[p] = ref["coords"]
    mesh = af.Mesh.from_arrays(ctx, dim, cells, coords)
    if order != "default":
        variant("AFEM_ORDER", order)
    bsr, ls = _assemble_gpu(ctx, mesh, 5.5)
    st = bsr.stats()
    if order == "default" and dim == 3:
        # bricks of the recovered lattice; a random numbering scatters each
        # row's sorted columns, so the bricks' slot streams differ row to row
        # (no uniform slices: the general instance runs them)
        assert st["brick_order"] == 2
    else:
        assert st["brick_order"] == 0
    if order != "default":
        variant("AFEM_ORDER", None)
    if order != "node":
        # the curve sort / brick order ran: a slice's rows are spatial
        # neighbours, so it couples to far fewer distinct nodes than 64 random
        # rows would
        m2 = af.Mesh.from_arrays(ctx, dim, cells, coords)
        variant("AFEM_ORDER", "node")
        b2, _ = _assemble_gpu(ctx, m2, 5.5)
        variant("AFEM_ORDER", None)
        assert st["max_slice_nodes"] < 0.6 * b2.stats()["max_slice_nodes"]
    rows, cols, vals = bsr.download()
    orp, ocols = O.sparsity(nn, nn, cells)
    ovals, orhs = O.assemble_poisson(nn, cells, coords, orp, ocols, 5.5)
    assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
    _check_values(vals, ovals)
    assert np.abs(ls.rhs_host() - orhs).max() <= VAL_TOL * np.abs(orhs).max()
    # against the unpermuted box: A_perm[p[i], p[j]] == A[i, j]
    m0 = af.Mesh.structured(ctx, dim, n, jitter=0.2, seed=20250220)
    b0, _ = _assemble_gpu(ctx, m0, 5.5)
    r0, c0, v0 = b0.download()
    A0 = {}
    for i in range(nn):
        for k in range(r0[i], r0[i + 1]):
            A0[(p[i], p[c0[k]])] = v0[k]
    scale = np.abs(v0).max()
    for i in range(nn):
        for k in range(rows[i], rows[i + 1]):
            assert abs(vals[k] - A0[(i, cols[k])]) <= VAL_TOL * scale


@pytest.mark.parametrize("n,nz,jitter", [(9, 9, 0.2), (14, 5, 0.0), (5, 23, 0.19)])
def test_lattice_order_matches_generator_box(ctx, variant, n, nz, jitter):
    """A generator box handed over as plain arrays in its own numbering: the
    recovered lattice gives the generator's brick order, the same stencil /
    uniform slice lists and bitwise the same matrix and RHS as the box made by
    afem_mesh_create_structured (unjittered and non-cubic boxes included)."""
    variant("AFEM_ASSEMBLY_CUBES", "0")  # the row-strip family (generator boxes default to cubes.hip)
    m0 = af.Mesh.structured(ctx, 3, n, nz=nz, jitter=jitter, seed=5)
    b0, l0 = _assemble_gpu(ctx, m0, 5.5)
    cells, coords, _ = m0.download()
    m1 = af.Mesh.from_arrays(ctx, 3, cells, coords)
    b1, l1 = _assemble_gpu(ctx, m1, 5.5)
    s0, s1 = b0.stats(), b1.stats()
    assert s0["brick_order"] == 1 and s1["brick_order"] == 2
    for k in ("n_slices", "uniform_slices", "stencil_slices", "stencil_sig", "max_slice_nodes"):
        assert s0[k] == s1[k], (k, s0[k], s1[k])
    r0, c0, v0 = b0.download()
    r1, c1, v1 = b1.download()
    assert np.array_equal(r0, r1) and np.array_equal(c0, c1)
    assert np.array_equal(v0, v1)
    assert np.array_equal(l0.rhs_host(), l1.rhs_host())


@pytest.mark.parametrize("n,nz,seed", [(12, 12, 77), (9, 17, 5), (6, 40, 3)])
def test_canonical_lattice_random_numbering(ctx, variant, n, nz, seed):
    """A generator box renumbered at random (nodes and cells) and handed over
    as arrays: the structure build relabels it by lattice index
    (sparsity.hip canonical_lattice), so its slices reach the same stencil /
    uniform instances as the generator's box, and the kernels store through
    the per-row slot map.  The matrix is bitwise the generator's, permuted
    (A1[p[i], p[j]] == A0[i, j]), and so is the RHS.  AFEM_CANON=0 (no
    relabeling: the general instance) stays within the oracle tolerance."""
    variant("AFEM_ASSEMBLY_CUBES", "0")  # the row-strip family (generator boxes default to cubes.hip)
    m0 = af.Mesh.structured(ctx, 3, n, nz=nz, jitter=0.2, seed=seed)
    b0, l0 = _assemble_gpu(ctx, m0, 5.5)
    cells0, coords0, _ = m0.download()
    rng = np.random.default_rng(seed)
    nn = coords0.shape[0]
    p = rng.permutation(nn)
    cells = p[cells0].astype(np.int32)[rng.permutation(cells0.shape[0])]
    coords = np.empty_like(coords0)
    coords[p] = coords0
    m1 = af.Mesh.from_arrays(ctx, 3, cells, coords)
    b1, l1 = _assemble_gpu(ctx, m1, 5.5)
    s0, s1 = b0.stats(), b1.stats()
    assert s1["brick_order"] == 2
    for k in ("n_slices", "uniform_slices", "stencil_slices", "stencil_sig"):
        assert s0[k] == s1[k], (k, s0[k], s1[k])
    assert s1["stencil_slices"] > 0
    r0, c0, v0 = b0.download()
    r1, c1, v1 = b1.download()
    key0 = p[np.repeat(np.arange(nn), np.diff(r0))].astype(np.int64) * nn + p[c0]
    key1 = np.repeat(np.arange(nn), np.diff(r1)).astype(np.int64) * nn + c1
    o0, o1 = np.argsort(key0), np.argsort(key1)
    assert np.array_equal(key0[o0], key1[o1])
    assert np.array_equal(v0[o0], v1[o1])
    assert np.array_equal(l1.rhs_host()[p], l0.rhs_host())
    # without the relabeling: the general instance, oracle tolerance
    variant("AFEM_CANON", "0")
    m2 = af.Mesh.from_arrays(ctx, 3, cells, coords)
    b2, _ = _assemble_gpu(ctx, m2, 5.5)
    variant("AFEM_CANON", None)
    assert b2.stats()["stencil_slices"] == 0
    r2, c2, v2 = b2.download()
    assert np.array_equal(r1, r2) and np.array_equal(c1, c2)
    _check_values(v2, v1)


@pytest.mark.parametrize("knobs", [{"AFEM_CUBES_YEX": "0"}, {"AFEM_CUBES_XEX": "0"},
                                   {"AFEM_CUBES_CARRY": "0", "AFEM_CUBES_STRIDE": "49"}])
def test_cube_kernel_face_sharing_variants(ctx, variant, knobs):
    """The cube kernel's face-sharing variants (y exchange off, x exchange off,
    no carry at 49-row planes) on a box with partial columns and z segments:
    the oracle's matrix and RHS (1e-12), the default's to rounding."""
    mesh = af.Mesh.structured(ctx, 3, 17, 11, jitter=0.2, seed=8)
    variant("AFEM_CUBES_ZS", "4")
    b0, l0 = _assemble_gpu(ctx, mesh, 5.5)
    v0, r0 = b0.download()[2], l0.rhs_host()
    for k, v in knobs.items():
        variant(k, v)
    b1, l1 = _assemble_gpu(ctx, mesh, 5.5)
    assert b1.stats()["last_kernel"] == 10
    rows, cols, v1 = b1.download()
    cells, coords, _ = mesh.download()
    orp, ocols = O.sparsity(mesh.n_nodes, mesh.n_own_nodes, cells)
    ovals, orhs = O.assemble_poisson(mesh.n_own_nodes, cells, coords, orp, ocols, 5.5)
    _check_values(v1, ovals)
    assert np.abs(l1.rhs_host() - orhs).max() <= VAL_TOL * np.abs(orhs).max()
    assert np.abs(v1 - v0).max() <= VAL_TOL * np.abs(v0).max()
    assert np.abs(l1.rhs_host() - r0).max() <= VAL_TOL * np.abs(r0).max()


@pytest.mark.parametrize("n,nz,seed", [(6, 6, 3), (9, 15, 4), (13, 5, 5), (1, 3, 6)])
def test_cube_kernel_on_random_numbering(ctx, n, nz, seed):
    """The cube kernel on a lattice of Kuhn cubes handed over as arrays in a
    random node and cell numbering (Structure::cube_*: the unit walks lattice
    indices, coordinates come through the caller's ids, each row's values go
    through its slot map): bitwise the generator box's matrix and RHS (also
    through the cube kernel), permuted; set and add RHS modes; the cells'
    vertex order does not matter (the kernel derives the cubes from the
    lattice).  Boxes too small for the canonical relabeling stay on the strip
    kernels (oracle tolerance)."""
    m0 = af.Mesh.structured(ctx, 3, n, nz=nz, jitter=0.2, seed=seed)
    b0, l0 = _assemble_gpu(ctx, m0, 5.5)
    assert b0.stats()["last_kernel"] == 10
    cells0, coords0, _ = m0.download()
    rng = np.random.default_rng(seed)
    nn = coords0.shape[0]
    p = rng.permutation(nn)
    cells = p[cells0].astype(np.int32)[rng.permutation(cells0.shape[0])]
    coords = np.empty_like(coords0)
    coords[p] = coords0
    m1 = af.Mesh.from_arrays(ctx, 3, cells, coords)
    b1, l1 = _assemble_gpu(ctx, m1, 5.5)
    if n >= 6:  # the canonical relabeling needs interior bricks (structure build)
        assert b1.stats()["last_kernel"] == 10
    r0, c0, v0 = b0.download()
    r1, c1, v1 = b1.download()
    key0 = p[np.repeat(np.arange(nn), np.diff(r0))].astype(np.int64) * nn + p[c0]
    key1 = np.repeat(np.arange(nn), np.diff(r1)).astype(np.int64) * nn + c1
    o0, o1 = np.argsort(key0), np.argsort(key1)
    assert np.array_equal(key0[o0], key1[o1])
    if b1.stats()["last_kernel"] == 10:
        assert np.array_equal(v0[o0], v1[o1])
        assert np.array_equal(l1.rhs_host()[p], l0.rhs_host())
    else:
        _check_values(v1[o1], v0[o0])
    rhs1 = l1.rhs_host()
    b1.assemblePoissonP1(1.0, 5.5, l1.rhsVariable(), rhs_mode="add")
    assert np.array_equal(l1.rhs_host(), rhs1 + rhs1)
    # another vertex order in every cell: the same cubes, the same bits
    cells2 = np.ascontiguousarray(cells[:, [2, 0, 3, 1]])
    m2 = af.Mesh.from_arrays(ctx, 3, cells2, coords)
    b2, _ = _assemble_gpu(ctx, m2, 5.5)
    assert b2.stats()["last_kernel"] == b1.stats()["last_kernel"]
    if b1.stats()["last_kernel"] == 10:
        assert np.array_equal(b2.download()[2], v1)
    else:
        _check_values(b2.download()[2], v1)


@pytest.mark.parametrize("n,nz,seed", [(6, 6, 3), (9, 15, 4), (13, 5, 5), (20, 7, 8)])
def test_cube_kernel_staged_canonical(ctx, variant, n, nz, seed):
    """The canonical cube path staged (V bit 1024: lattice-order 128-B lines,
    then k_cube_unstage into the caller's rows) against the single-pass
    canonical flush: the same matrix and RHS bits, set and add RHS modes, an
    assembly repeated on the same structure (maps and stage built once)."""
    m0 = af.Mesh.structured(ctx, 3, n, nz=nz, jitter=0.2, seed=seed)
    cells0, coords0, _ = m0.download()
    rng = np.random.default_rng(seed)
    nn = coords0.shape[0]
    p = rng.permutation(nn)
    cells = p[cells0].astype(np.int32)[rng.permutation(cells0.shape[0])]
    coords = np.empty_like(coords0)
    coords[p] = coords0
    m1 = af.Mesh.from_arrays(ctx, 3, cells, coords)
    out = {}
    for staged in (False, True):
        variant("AFEM_CUBES_V", None if staged else str(CUBES_V & ~1024))
        b1, l1 = _assemble_gpu(ctx, m1, 5.5)
        assert b1.stats()["last_kernel"] == 10
        rhs = l1.rhs_host()
        b1.assemblePoissonP1(1.0, 5.5, l1.rhsVariable(), rhs_mode="add")
        added = l1.rhs_host()
        b1.resetMatrixValues()
        b1.assemblePoissonP1(2.0)  # no RHS: the matrix alone (k_cube_unstage<false, false>)
        out[staged] = (b1.download(), rhs, added)
    (r0, c0, v0), s0, a0 = out[False]
    (r1, c1, v1), s1, a1 = out[True]
    assert np.array_equal(r0, r1) and np.array_equal(c0, c1)
    assert np.array_equal(v0, v1)
    assert np.array_equal(s0, s1)
    assert np.array_equal(a0, a1)


AXIS_ORDERS = [(0, 1, 2), (0, 2, 1), (1, 0, 2), (1, 2, 0), (2, 0, 1), (2, 1, 0)]


def natural_numbering(n, nz, order):
    """New id of every generator node (id = x + (n+1)(y + (n+1) z)) when the
    box is numbered lexicographically with the axes in `order`, fastest first
    (Arcane's cartesian generator: x fastest = (0, 1, 2))."""
    L = np.array([n + 1, n + 1, nz + 1], dtype=np.int64)
    ids = np.arange(L.prod(), dtype=np.int64)
    lat = np.stack([ids % L[0], (ids // L[0]) % L[1], ids // (L[0] * L[1])])
    a, b, c = order
    return lat[a] + L[a] * (lat[b] + L[b] * lat[c])


@pytest.mark.parametrize("order", AXIS_ORDERS)
@pytest.mark.parametrize("n,nz,seed", [(9, 15, 4), (13, 6, 5)])
def test_cube_kernel_on_natural_numbering(ctx, variant, n, nz, seed, order):
    """a lattice of Kuhn cubes handed over as arrays in a
    NATURAL numbering (lexicographic in any axis order, cells in a random
    order, vertices in any order) runs the headline cube kernel with no map
    (cube_lattice 2).  The caller's structure and the oracle's on the same
    arrays are equal, the values and RHS within 1e-12; for x-fastest order the
    matrix is bitwise the generator box's; AFEM_CUBE_NATURAL=0 (the strip
    kernels) agrees to rounding."""
    m0 = af.Mesh.structured(ctx, 3, n, nz=nz, jitter=0.2, seed=seed)
    b0, l0 = _assemble_gpu(ctx, m0, 5.5)
    cells0, coords0, _ = m0.download()
    rng = np.random.default_rng(seed)
    p = natural_numbering(n, nz, order)
    cells = p[cells0].astype(np.int32)[rng.permutation(cells0.shape[0])]
    cells = np.ascontiguousarray(np.take_along_axis(cells, rng.permuted(np.tile(np.arange(4), (cells.shape[0], 1)),
                                                                        axis=1), axis=1))
    coords = np.empty_like(coords0)
    coords[p] = coords0
    m1 = af.Mesh.from_arrays(ctx, 3, cells, coords)
    b1, l1 = _assemble_gpu(ctx, m1, 5.5)
    st = b1.stats()
    assert st["cube_lattice"] == 2 and st["last_kernel"] == 10, st
    assert st["cube_axes"] == order[0] + 3 * order[1] + 9 * order[2]
    rows, cols, vals = b1.download()
    rhs = l1.rhs_host()
    orp, ocols = O.sparsity(m1.n_nodes, m1.n_own_nodes, cells)
    ovals, orhs = O.assemble_poisson(m1.n_own_nodes, cells, coords, orp, ocols, 5.5)
    assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
    _check_values(vals, ovals)
    assert np.abs(rhs - orhs).max() <= VAL_TOL * np.abs(orhs).max()
    if order == (0, 1, 2):
        assert np.array_equal(vals, b0.download()[2]) and np.array_equal(rhs, l0.rhs_host())
    variant("AFEM_CUBE_NATURAL", "0")
    m2 = af.Mesh.from_arrays(ctx, 3, cells, coords)
    b2, l2 = _assemble_gpu(ctx, m2, 5.5)
    assert b2.stats()["cube_lattice"] != 2
    _check_values(b2.download()[2], vals)
    assert np.abs(l2.rhs_host() - rhs).max() <= VAL_TOL * np.abs(rhs).max()


def test_natural_numbering_rejects_non_kuhn_lattices(ctx):
    """A lattice whose cubes are not cut into the 6 Kuhn tets (here: one cube's
    tets replaced by the other diagonal's) or whose numbering is not
    lexicographic stays off the natural path, with the oracle's matrix."""
    n = 6
    m0 = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=2)
    cells0, coords0, _ = m0.download()
    # a node swap breaks the lexicographic numbering
    p = np.arange(coords0.shape[0])
    p[[5, 40]] = p[[40, 5]]
    cells = p[cells0].astype(np.int32)
    coords = np.empty_like(coords0)
    coords[p] = coords0
    for cc in (cells, None):
        if cc is None:
            # cube 0's six tets re-cut along the diagonal (1,0,0)-(0,1,1)
            L = n + 1
            v = lambda x, y, z: x + L * (y + L * z)  # noqa: E731
            cc = cells0.copy()
            # the monotone paths from (1,0,0) to (0,1,1) (x reflected)
            six = [[v(1, 0, 0), v(0, 0, 0), v(0, 1, 0), v(0, 1, 1)], [v(1, 0, 0), v(0, 0, 0), v(0, 0, 1), v(0, 1, 1)],
                   [v(1, 0, 0), v(1, 1, 0), v(0, 1, 0), v(0, 1, 1)], [v(1, 0, 0), v(1, 1, 0), v(1, 1, 1), v(0, 1, 1)],
                   [v(1, 0, 0), v(1, 0, 1), v(0, 0, 1), v(0, 1, 1)], [v(1, 0, 0), v(1, 0, 1), v(1, 1, 1), v(0, 1, 1)]]
            cube0 = np.where(np.all(np.isin(cc, [v(x, y, z) for x in (0, 1) for y in (0, 1) for z in (0, 1)]), axis=1))[0]
            assert cube0.size == 6
            cc[cube0] = np.array(six, dtype=np.int32)
            crd = coords0
        else:
            crd = coords
        m1 = af.Mesh.from_arrays(ctx, 3, cc, crd)
        b1, l1 = _assemble_gpu(ctx, m1, 5.5)
        assert b1.stats()["cube_lattice"] != 2
        rows, cols, vals = b1.download()
        orp, ocols = O.sparsity(m1.n_nodes, m1.n_own_nodes, cc)
        ovals, orhs = O.assemble_poisson(m1.n_own_nodes, cc, crd, orp, ocols, 5.5)
        assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
        _check_values(vals, ovals)


@pytest.mark.parametrize("knob,value", [("AFEM_BANK_PLACE_GENERAL", "1"), ("AFEM_ASSEMBLY_LOCAL", "1"),
                                        ("AFEM_ASSEMBLY_BIG", "0"), ("AFEM_ASSEMBLY_BIG", "1")])
def test_general_slice_variants_bitwise(ctx, variant, knob, value):
    """Variants of the general (unstructured) slices that must not change a
    bit: LDS-bank-aware placement of their node lists (a greedy colouring of
    the positions mod 32 over the lanes that read them at each step,
    sparsity.hip bank_place_general; opt-in), the local-index stream
    instead of the column-index table (AFEM_ASSEMBLY_LOCAL=1: the slices of
    <= 256 nodes through k_assemble_strip<4,2,16,3>; opt-in), and the order of
    the compact and big lists (AFEM_ASSEMBLY_BIG 0: side by side, 1: big
    first; the default compact first).  On an unstructured mesh: the matrix and
    the RHS bitwise equal to the default's, and the oracle's."""
    import bench

    gm = read_gmsh(path("L-shape-3D.msh"))
    cells, coords = bench.refine_tets(gm.cells, gm.coords, 3, "cpu")  # 25.6 k nodes, 133 k tets
    out = {}
    for mode in ("default", "variant"):
        variant(knob, value if mode == "variant" else None)
        mesh = af.Mesh.from_arrays(ctx, 3, cells, coords)
        bsr, ls = _assemble_gpu(ctx, mesh, 5.5)
        st = bsr.stats()
        assert st["general_slices"] > 0 and st["brick_order"] == 0
        out[mode] = (bsr.download(), ls.rhs_host())
    (r0, c0, v0), h0 = out["default"]
    (r1, c1, v1), h1 = out["variant"]
    assert np.array_equal(r0, r1) and np.array_equal(c0, c1)
    assert np.array_equal(v0, v1) and np.array_equal(h0, h1)
    n = coords.shape[0]
    orp, ocols = O.sparsity(n, n, cells)
    ovals, orhs = O.assemble_poisson(n, cells, coords, orp, ocols, 5.5)
    assert np.array_equal(r0, orp) and np.array_equal(c0, ocols)
    _check_values(v0, ovals)


def test_lattice_order_rejects_non_lattices(ctx):
    """Coordinates that are not a lattice (a Kuhn box whose node layers are
    warped beyond the gap rule, and one missing node) fall back to the
    Hilbert order; the values stay the oracle's."""
    ref = O.structured_mesh(3, 8, jitter=0.2, seed=9)
    coords = ref["coords"].copy()
    coords[:, 0] += 0.9 * (coords[:, 1] ** 2)  # shear the x layers into each other
    mesh = af.Mesh.from_arrays(ctx, 3, ref["cells"], coords)
    bsr, ls = _assemble_gpu(ctx, mesh, 5.5)
    assert bsr.stats()["brick_order"] == 0
    rows, cols, vals = bsr.download()
    orp, ocols = O.sparsity(ref["n_local"], ref["n_local"], ref["cells"])
    ovals, _ = O.assemble_poisson(ref["n_local"], ref["cells"], coords, orp, ocols, 5.5)
    assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
    _check_values(vals, ovals)
    # drop the cells of node 0's corner: node 0 is isolated but still a lattice point;
    # drop node count instead: the last node removed -> layer product != n_rows
    keep = ~(ref["cells"] == ref["n_local"] - 1).any(axis=1)
    m2 = af.Mesh.from_arrays(ctx, 3, ref["cells"][keep], ref["coords"][:-1])
    b2, _ = _assemble_gpu(ctx, m2, 5.5)
    assert b2.stats()["brick_order"] == 0


@pytest.mark.parametrize("dim", [2, 3])
def test_mesh_without_cells(ctx, dim):
    # nodes but no cells: every row is its diagonal alone (BSRFormat.h:679 always
    # inserts it), all values and the RHS are zero
    coords = np.random.default_rng(3).random((70, 3))
    if dim == 2:
        coords[:, 2] = 0.0
    cells = np.zeros((0, dim + 1), dtype=np.int32)
    mesh = af.Mesh.from_arrays(ctx, dim, cells, coords)
    bsr, ls = _assemble_gpu(ctx, mesh, 5.5)
    rows, cols, vals = bsr.download()
    assert np.array_equal(rows, np.arange(71)) and np.array_equal(cols, np.arange(70))
    assert not vals.any() and not ls.rhs_host().any()


@pytest.mark.parametrize("dim", [2, 3])
def test_single_cell(ctx, dim):
    coords = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0.2, 0.3, 1.1]], dtype=np.float64)[: dim + 1]
    cells = np.arange(dim + 1, dtype=np.int32)[None, :]
    mesh = af.Mesh.from_arrays(ctx, dim, cells, coords)
    bsr, ls = _assemble_gpu(ctx, mesh, 2.0)
    rows, cols, vals = bsr.download()
    orp, ocols = O.sparsity(dim + 1, dim + 1, cells)
    ovals, orhs = O.assemble_poisson(dim + 1, cells, coords, orp, ocols, 2.0)
    assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
    _check_values(vals, ovals)
    assert np.abs(ls.rhs_host() - orhs).max() <= VAL_TOL * np.abs(orhs).max()


def test_c_driver_through_the_c_abi(ctx, tmp_path):
    # examples/poisson3d.c runs the Poisson module's sequence through the C ABI
    # alone; its solution equals the one of the same calls made from Python
    import os
    import subprocess

    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "poisson3d")
    assert os.path.exists(exe), "examples/poisson3d not built (make -C examples)"
    out = tmp_path / "u.bin"
    res = subprocess.run([exe, "8", str(out)], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stderr
    assert "converged=1" in res.stdout, res.stdout
    u_c = np.fromfile(out, dtype=np.float64)
    mesh = af.Mesh.structured(ctx, 3, 8, jitter=0.2, seed=20250220)
    bsr, ls = _assemble_gpu(ctx, mesh, 5.5)
    ls.applyDirichletViaPenalty(mesh.bottom_nodes(), 0.5, 1e30)
    ls.setSolverOptions(rtol=1e-13)
    ls.solve()
    u_py = ls.solution_host()[: mesh.n_own_nodes]
    assert u_c.shape == u_py.shape
    assert np.abs(u_c - u_py).max() <= 1e-12 * np.abs(u_py).max()
    cells, coords, _ = mesh.download()
    orp, ocols = O.sparsity(mesh.n_nodes, mesh.n_own_nodes, cells)
    ovals, orhs = O.assemble_poisson(mesh.n_own_nodes, cells, coords, orp, ocols, 5.5)
    O.dirichlet_penalty(mesh.bottom_nodes(), 0.5, 1e30, orp, ocols, ovals, orhs)
    xo = np.linalg.solve(O.csr_to_dense(orp, ocols, ovals), orhs)
    assert np.abs(u_c - xo).max() <= SOL_TOL * np.abs(xo).max()


def test_rccl_communicator_single_rank(ctx):
    # the RCCL data path of bench.py --gpus N at N = 1: communicator bootstrap
    # (ncclGetUniqueId / ncclCommInitRank), halo plan of the slab layout, solve
    # with the halo attached (exchange and all-reduce are identities on one
    # rank) equals the solve without it.  N > 1 needs one GPU per rank (RCCL
    # refuses two ranks on one device); its decomposition logic is covered on
    # CPU by tests/test_distributed_gloo.py.
    mesh = af.Mesh.structured(ctx, 3, 10, jitter=0.2, seed=20250220)
    uid = af.Communicator.unique_id()
    comm = af.Communicator(ctx, 1, 0, uid)
    try:
        sols = []
        for with_halo in (False, True):
            bsr, ls = _assemble_gpu(ctx, mesh, 5.5)
            if with_halo:
                ls.set_halo_structured(comm, mesh)
            ls.applyDirichletViaPenalty(mesh.bottom_nodes(), 0.5, 1e30)
            ls.setSolverOptions(rtol=1e-12)
            st = ls.solve()
            assert st["converged"]
            sols.append(ls.solution_host()[: mesh.n_own_nodes])
        assert np.array_equal(sols[0], sols[1])
    finally:
        comm.close()


def test_initial_guess_current_solution(ctx):
    """afem_solver_opts::initial_guess = 1 starts the PCG from the solution
    vector: from the converged solution it stops at once with the same
    answer; from a perturbed one it converges to the cold-start solution
    (same stopping target: the zero guess's residual)."""
    gm = read_gmsh(path("sphere_cut.msh"))
    mesh = af.Mesh.from_arrays(ctx, gm.dim, gm.cells, gm.coords)
    bsr, ls = _assemble_gpu(ctx, mesh, 5.5)
    ls.applyDirichletViaPenalty(gm.group_nodes("horizontal"), 0.5, 1e30)
    ls.setSolverOptions(rtol=1e-12, max_iter=20000, method="pcg", initial_guess="zero")
    st0 = ls.solve()
    x0 = ls.solution_host()
    ls.setSolverOptions(initial_guess="current")
    st1 = ls.solve()
    assert st1["converged"] and st1["iterations"] <= 8
    assert np.abs(ls.solution_host() - x0).max() <= 1e-12 * np.abs(x0).max()
    pert = x0 * (1.0 + 1e-3 * np.sin(np.arange(x0.size)))
    ctx.to_device(ls.solutionVariable(), pert)
    st2 = ls.solve()
    assert st2["converged"] and st2["iterations"] < st0["iterations"]
    assert np.abs(ls.solution_host() - x0).max() <= 1e-9 * np.abs(x0).max()
    ls.setSolverOptions(initial_guess="zero")


@pytest.mark.parametrize("n", [9, 30])
def test_pattern_spmv(ctx, variant, n):
    """The pattern-compressed SpMV (interior rows of a Kuhn box form their
    columns as row + the offsets of the interior stencil, the others read
    theirs, into the block's LDS column image): the same products in the same
    order as the CSR-stream kernel (bitwise equal y), and the same CG solve."""
    mesh = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=5)
    bsr, ls = _assemble_gpu(ctx, mesh, 5.5)
    bottom = mesh.bottom_nodes()
    ls.applyDirichletViaPenalty(bottom, 0.5, 1.0e30)
    ls.applyBoundaryConditions()
    nn = mesh.n_own_nodes
    x = np.random.default_rng(3).standard_normal(nn)
    dx, dy = ctx.malloc(8 * nn), ctx.malloc(8 * nn)
    ctx.to_device(dx, x)
    ys = {}
    for mode in ("nopat", "pat"):
        variant("AFEM_SPMV", mode)
        ls.spmv(dx, dy)
        ys[mode] = ctx.to_host(dy, nn, np.float64)
    ctx.free(dx)
    ctx.free(dy)
    assert np.array_equal(ys["nopat"], ys["pat"])
    sols, kern = {}, {}
    for mode in ("nopat", "pat", None):
        if mode is None:
            variant("AFEM_SPMV", None)  # the default: the pattern kernel, 64-row blocks
            variant("AFEM_SPMV_BS", None)
        else:
            variant("AFEM_SPMV", mode)
            variant("AFEM_SPMV_BS", "256")  # the CSR-stream kernel's blocks: the same partial sums
        kern[mode] = ls.solve()["spmv_kernel"]
        sols[mode] = ls.solution_host()
    assert kern == {"nopat": 0, "pat": 1, None: 1}, kern
    assert np.array_equal(sols["nopat"], sols["pat"])
    # 64-row blocks: the same y; the dot products' block partials are summed in
    # another grouping, so the iterates agree to rounding
    assert np.abs(sols["pat"] - sols[None]).max() <= 1e-12 * np.abs(sols["pat"]).max()


@pytest.mark.parametrize("rank", [0, 1, 2])
def test_stencil_on_slab_subdomains(ctx, rank):
    """z-slab subdomains (owned layers + one ghost layer, ghosts numbered
    after the owned nodes): the interior bricks still match the compiled-in
    signatures; the slab's assembly against the oracle on the same subdomain."""
    mesh = af.Mesh.structured(ctx, 3, 20, nz=36, jitter=0.2, seed=9, nranks=3, rank=rank)
    bsr, ls = _assemble_gpu(ctx, mesh, 2.5)
    st = bsr.stats()
    assert st["stencil_slices"] > 0, st
    rows, cols, vals = bsr.download()
    cells, coords, _ = mesh.download()
    orp, ocols = O.sparsity(mesh.n_nodes, mesh.n_own_nodes, cells)
    ovals, orhs = O.assemble_poisson(mesh.n_own_nodes, cells, coords, orp, ocols, 2.5)
    assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
    _check_values(vals, ovals)
    assert np.abs(ls.rhs_host() - orhs).max() <= VAL_TOL * np.abs(orhs).max()


@pytest.mark.parametrize("mode", [dict(rtol=1e-13), dict(fixed_iterations=37)])
def test_cg_graph_replay_bitwise(ctx, variant, mode):
    """With AFEM_CG_GRAPH=1 the single-rank CG replays whole iterations as a
    captured HIP graph (batches of the convergence-check period / 16 fixed
    iterations; opt-in, slower than launching on MI355X); it must run exactly
    the launches of the per-kernel loop (the default): the same iteration
    count and the same solution bits."""
    mesh = af.Mesh.structured(ctx, 3, 17, jitter=0.2, seed=3)
    bsr, ls = _assemble_gpu(ctx, mesh, 5.5)
    ls.applyDirichletViaPenalty(mesh.bottom_nodes(), 0.5, 1e30)
    out = []
    for g in ("1", None):
        variant("AFEM_CG_GRAPH", g)
        ls.setSolverOptions(**mode)
        st = ls.solve()
        out.append((st["iterations"], ls.solution_host()))
    assert out[0][0] == out[1][0]
    assert np.array_equal(out[0][1], out[1][1])


@pytest.mark.parametrize("pc", ["jacobi", "amg"])
def test_rccl_self_loop_solve(ctx, variant, pc):
    """The RCCL data path on ONE GPU (AFEM_COMM_SELF=1: a one-rank communicator
    runs its collectives, a halo may name the own rank): the sphere's Poisson
    system with 40 owned DoFs also addressed as ghost columns (half of their
    couplings in the CSR go to the ghost alias, whose value the halo's
    ncclSend / ncclRecv to self fills), solved by the distributed PCG -- the
    split SpMV with the exchange on the halo stream, ncclAllReduce of the
    scalars, and for pc = amg the distributed AMG (aggregation ghost-blind,
    coarse ghost columns and halo, the gathered level) -- equals the plain
    system's solution.  What the driver's 8-GPU run executes, minus the
    second device."""
    variant("AFEM_COMM_SELF", "1")
    if pc == "amg":
        variant("AFEM_AMG_DENSE", "16")
    gm = read_gmsh(path("sphere_cut.msh"))
    n = gm.n_nodes
    rp, cols = O.sparsity(n, n, gm.cells)
    vals, rhs = O.assemble_poisson(n, gm.cells, gm.coords, rp, cols, 5.5)
    dn = gm.group_nodes("horizontal")
    O.dirichlet_penalty(dn, 0.5, 1e30, rp, cols, vals, rhs)
    rng = np.random.default_rng(40)
    S = np.sort(rng.choice(n, 40, replace=False)).astype(np.int32)
    alias = {int(s): n + k for k, s in enumerate(S)}
    gcols = cols.copy()
    gvals = vals.copy()
    for i in range(n):
        seg = slice(rp[i], rp[i + 1])
        c = np.array([alias[int(x)] if (int(x) in alias and int(x) != i and i % 2 == 0) else int(x)
                      for x in cols[seg]], dtype=np.int32)
        o = np.argsort(c, kind="stable")
        gcols[seg] = c[o]
        gvals[seg] = vals[seg][o]
    assert (gcols >= n).sum() > 40
    uid = af.Communicator.unique_id()
    comm = af.Communicator(ctx, 1, 0, uid)
    try:
        sols, its = [], []
        for ghosts in (False, True):
            ls = af.DoFLinearSystem().initialize(ctx, n, n + 40)
            if ghosts:
                ls.setCSRValues(rp[:-1].astype(np.int32), None, gcols, gvals)
                ls.set_halo(comm, [0], [S], [np.arange(n, n + 40, dtype=np.int32)])
            else:
                ls.setCSRValues(rp[:-1].astype(np.int32), None, cols, vals)
            ls.set_rhs_host(rhs)
            ls.setSolverOptions(rtol=1e-13, max_iter=20000, method="pcg", preconditioner=pc)
            st = ls.solve()
            assert st["converged"], (ghosts, st)
            sols.append(ls.solution_host().copy())
            its.append(st["iterations"])
            if ghosts:
                assert st["n_allreduce"] > 0 and st["n_halo"] > 0  # the RCCL calls ran
            ls.reset()
        xo = np.linalg.solve(O.csr_to_dense(rp, cols, vals), rhs)
        for x in sols:
            assert np.abs(x - xo).max() <= 1e-10 * np.abs(xo).max()
        print(f"\nRCCL self loop, {pc}: iterations plain / with the self halo {its}")
    finally:
        comm.close()
