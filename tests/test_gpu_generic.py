"""GPU: BSRFormat::assembleBilinear(lambda) through the generic element-functor
entry (include/arcanefem_amd_generic.hpp) -- the module's own element functor
(a hipcc-compiled device lambda, examples/generic_assembly.hip) evaluated once
per (unit, cell) by the cell-unit kernel k_assemble_units (rows of a unit in
LDS, wavefront-local ds_add_f64 in program order, no global atomics: bitwise
reproducible), and by the reference's own algorithm (one lane per cell, f64
atomics into HBM, femutils/BSRFormat.h:786-837: assemble_bilinear_atomic).

Gates per entry (summation order differs from the fixed-physics strip
kernels, as the reference's atomics differ run to run): against the library's
compiled-in instance on the same structure and against the oracle's cell loop
(orc_assemble_poisson / orc_assemble_elasticity_tet), |a - b| <= 1e-12 max|b|,
both value layouts (ordered per block, per row)."""
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "generic_assembly")


def _run(n, k, layout, tmp_path):
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} is not built (make -C examples)")
    out = str(tmp_path / f"g{n}_{k}_{layout}.bin")
    r = subprocess.run([EXE, str(n), str(k), layout, out], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = open(out, "rb").read()
    n_rows, nnz = np.frombuffer(raw[:16], dtype=np.int64)
    off = 16
    rows = np.frombuffer(raw[off:off + 8 * (n_rows + 1)], dtype=np.int64)
    off += 8 * (n_rows + 1)
    cols = np.frombuffer(raw[off:off + 4 * nnz], dtype=np.int32)
    off += 4 * nnz
    m = nnz * k * k
    gen = np.frombuffer(raw[off:off + 8 * m], dtype=np.float64)
    bi = np.frombuffer(raw[off + 8 * m:off + 16 * m], dtype=np.float64)
    return rows, cols, gen, bi


@pytest.mark.parametrize("layout", ["block", "row"])
@pytest.mark.parametrize("k", [1, 3])
def test_generic_lambda_matches_oracle(tmp_path, k, layout):
    n = 6
    rows, cols, gen, bi = _run(n, k, layout, tmp_path)
    ref = O.structured_mesh(3, n, jitter=0.2, seed=20250220)
    orp, ocols = O.sparsity(ref["n_local"], ref["n_own"], ref["cells"])
    assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
    if k == 1:
        ovals, _ = O.assemble_poisson(ref["n_own"], ref["cells"], ref["coords"], orp, ocols, 0.0)
    else:
        E, nu = 21.0e5, 0.28
        lam, mu = E * nu / ((1 + nu) * (1 - 2 * nu)), E / (2 * (1 + nu))
        ovals, _ = O.assemble_elasticity_tet(ref["n_own"], ref["cells"], ref["coords"], orp, ocols, lam, 2 * mu)
        if layout == "row":
            ovals = O.blocks_to_row_order_k(orp, ovals, 3)
    scale = np.abs(ovals).max()
    assert np.abs(gen - ovals).max() <= 1e-12 * scale, np.abs(gen - ovals).max() / scale
    assert np.abs(bi - ovals).max() <= 1e-12 * scale
    assert np.abs(gen - bi).max() <= 1e-12 * scale


# ---------------------------------------------------------------- the cell-unit kernel through ctypes
# examples/libafem_generic_example.so: the reference modules' element functors
# (examples/elements.hpp) through afem::generic::assemble_bilinear on any
# structure libafem builds -- lattice columns (generator boxes, slabs with
# ghost layers, array-fed lattices in a random numbering) and slice pieces
# (unstructured Gmsh meshes, 2D).  Gates: the oracle's cell loop and the
# atomic kernel per entry at 1e-12 of the largest value; the unit kernel is
# bitwise reproducible and Accumulate after Overwrite gives exactly twice the
# values.
import sys

sys.path.insert(0, os.path.join(ROOT, "examples"))

E_, NU_ = 21.0e5, 0.28
LAM_, MU_ = E_ * NU_ / ((1 + NU_) * (1 - 2 * NU_)), E_ / (2 * (1 + NU_))


def _random_numbering(n, seed=1234):
    ref = O.structured_mesh(3, n, jitter=0.2, seed=20250220)
    rng = np.random.default_rng(seed)
    nn = ref["coords"].shape[0]
    perm = rng.permutation(nn).astype(np.int32)
    coords = np.empty_like(ref["coords"])
    coords[perm] = ref["coords"]
    cells = perm[ref["cells"]]
    cells = cells[rng.permutation(cells.shape[0])]
    return np.ascontiguousarray(cells, dtype=np.int32), coords


def _mesh(ctx, which):
    import arcanefem_amd as af
    from arcanefem_amd.gmsh import read_gmsh

    from golden_cases import path

    if which == "box":
        return af.Mesh.structured(ctx, 3, 12, jitter=0.2, seed=20250220)
    if which == "slab":
        return af.Mesh.structured(ctx, 3, 10, jitter=0.2, seed=20250220, nranks=3, rank=1)
    if which == "arrays_random":
        cells, coords = _random_numbering(11)
        return af.Mesh.from_arrays(ctx, 3, cells, coords)
    gm = read_gmsh(path({"sphere": "sphere_cut.msh", "lshape3d": "L-shape-3D.msh", "circle": "circle_cut.msh",
                         "bar": "bar.msh"}[which]))
    return af.Mesh.from_arrays(ctx, gm.dim, gm.cells, gm.coords)


def _oracle(mesh, k, per_row):
    cells, coords, _ = mesh.download()
    orp, ocols = O.sparsity(mesh.n_nodes, mesh.n_own_nodes, cells)
    if k == 1:
        ov, _ = O.assemble_poisson(mesh.n_own_nodes, cells, coords, orp, ocols, 0.0)
    elif k == 2:
        ov = O.assemble_elasticity_tri(mesh.n_own_nodes, cells, coords, orp, ocols, LAM_, 2 * MU_)
    else:
        ov, _ = O.assemble_elasticity_tet(mesh.n_own_nodes, cells, coords, orp, ocols, LAM_, 2 * MU_)
    if k > 1 and per_row:
        ov = O.blocks_to_row_order_k(orp, ov, k)
    return orp, ocols, ov


def _unit_case(ctx, mesh, k, per_row):
    import arcanefem_amd as af
    import generic_example as gx

    kind = gx.POISSON if k == 1 else gx.ELASTICITY
    bsr = af.BSRFormat(mesh, k).initialize(per_row)
    bsr.computeSparsity()
    gx.assemble(bsr, kind, gx.UNITS, overwrite=True, lam=LAM_, mu=MU_)
    rows, cols, a = bsr.download()
    gx.assemble(bsr, kind, gx.UNITS, overwrite=True, lam=LAM_, mu=MU_)
    a2 = bsr.download()[2]
    gx.assemble(bsr, kind, gx.UNITS, overwrite=False, lam=LAM_, mu=MU_)
    twice = bsr.download()[2]
    gx.assemble(bsr, kind, gx.ATOMIC, overwrite=True, lam=LAM_, mu=MU_)
    b = bsr.download()[2]
    plan = bsr.functor_plan()
    orp, ocols, ov = _oracle(mesh, k, per_row)
    assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
    sc = np.abs(ov).max()
    assert np.abs(a - ov).max() <= 1e-12 * sc, np.abs(a - ov).max() / sc
    assert np.abs(a - b).max() <= 1e-12 * sc, np.abs(a - b).max() / sc
    assert np.array_equal(a, a2), "the cell-unit kernel is not reproducible"
    assert np.array_equal(twice, 2.0 * a), "Accumulate did not add to the values"
    bsr.close()
    return plan


@pytest.mark.parametrize("per_row", [False, True])
@pytest.mark.parametrize("which,k,lattice", [("box", 1, 1), ("box", 3, 1), ("slab", 1, 1), ("slab", 3, 1),
                                             ("arrays_random", 1, 1), ("arrays_random", 3, 1), ("sphere", 1, 0),
                                             ("sphere", 3, 0), ("lshape3d", 1, 0), ("circle", 1, 0),
                                             ("bar", 2, 0)])
def test_unit_kernel_matches_oracle(ctx, which, k, lattice, per_row):
    mesh = _mesh(ctx, which)
    plan = _unit_case(ctx, mesh, k, per_row)
    assert plan["lattice"] == lattice, plan
    assert plan["block_size"] == k
    # every cell incident to an owned row is evaluated at least once per unit it touches
    assert plan["n_entries"] >= mesh.n_cells if which not in ("slab",) else plan["n_entries"] > 0
    mesh.close()


def test_unit_kernel_slice_plan_on_a_box(ctx, variant):
    """The single-layer slice plan (what non-lattice meshes get) on a lattice
    box gives the same values as the lattice columns (to rounding: the
    summation order differs)."""
    variant("AFEM_FUNCTOR_PLAN", "slices")
    mesh = _mesh(ctx, "box")
    plan = _unit_case(ctx, mesh, 1, True)
    assert plan["lattice"] == 0 and plan["nbuf"] == 1
    mesh.close()


@pytest.mark.parametrize("n", [3, 7])
def test_unit_kernel_slice_plan_partial_last_piece(ctx, variant, n):
    """k = 3 slice pieces hold 7 rows: 64 positions per slice do not divide
    into them, and the last piece of the structure is partial.  A box of
    (n + 1)^3 = 64 / 512 nodes fills its slices to the last lane, so the last
    piece holds an active row (it was dropped when the piece count was
    rounded down)."""
    import arcanefem_amd as af

    variant("AFEM_FUNCTOR_PLAN", "slices")
    mesh = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=3)
    assert mesh.n_own_nodes % 64 == 0
    for per_row in (False, True):
        plan = _unit_case(ctx, mesh, 3, per_row)
        assert plan["lattice"] == 0 and plan["rows_per_layer"] == 7
        assert plan["n_units"] * 7 >= mesh.n_own_nodes
    mesh.close()


def test_unit_kernel_evaluations_per_cell(ctx, variant):
    """The lattice columns evaluate each cell at most 1 + 1/8 + 1/8 + 1/zs
    times (the cells shared with the neighbour columns / segments; fewer at
    the box boundary)."""
    import arcanefem_amd as af

    variant("AFEM_FUNCTOR_ZS", "16")
    mesh = af.Mesh.structured(ctx, 3, 63, jitter=0.2, seed=20250220)
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    bsr.computeSparsity()
    plan = bsr.functor_plan()
    ratio = plan["n_entries"] / mesh.n_cells
    assert plan["lattice"] == 1 and plan["rows_per_layer"] == 64 and plan["nbuf"] == 2
    assert ratio < 1.0 + 1 / 8 + 1 / 8 + 1 / 16, ratio
    bsr.close()
    mesh.close()


@pytest.mark.parametrize("which,k", [("box", 1), ("box", 3), ("slab", 1), ("arrays_random", 1), ("sphere", 1)])
def test_packed_entries_bitwise(ctx, variant, which, k):
    """Packed plan entries (8 B {cell, pattern} + the table of distinct slot /
    position words) give the bits of the 16-B entries: the same cells in the
    same order, the same LDS adds.  Forced on (AFEM_FUNCTOR_PACKED=1: the
    format is opt-in, and small meshes' boundary rows make many patterns)."""
    import arcanefem_amd as af
    import generic_example as gx

    kind = gx.POISSON if k == 1 else gx.ELASTICITY
    vals = {}
    for pk in ("0", "1"):
        variant("AFEM_FUNCTOR_PACKED", pk)
        mesh = _mesh(ctx, which)
        bsr = af.BSRFormat(mesh, k).initialize(True)
        bsr.computeSparsity()
        plan = bsr.functor_plan()
        assert plan["packed"] == (1 if pk == "1" and not plan["wide"] else 0), plan
        if plan["packed"]:
            assert 0 < plan["n_patterns"] <= plan["n_entries"]
        gx.assemble(bsr, kind, gx.UNITS, overwrite=True, lam=LAM_, mu=MU_)
        vals[pk] = bsr.download()[2]
        if pk == "1":
            _, _, ov = _oracle(mesh, k, True)
            sc = np.abs(ov).max()
            assert np.abs(vals[pk] - ov).max() <= 1e-12 * sc
        bsr.close()
        mesh.close()
    assert np.array_equal(vals["0"], vals["1"])
