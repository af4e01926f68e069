"""CPU: pin the oracle against the reference's golden result files, and check
the oracle's own building blocks against known answers."""
import numpy as np
import pytest

from arcanefem_amd.gmsh import read_gmsh, read_node_result_file
from oracle import oracle as O

from golden_cases import CASES, GOLDEN_TOL, path


@pytest.mark.parametrize("case", list(CASES))
def test_oracle_reproduces_reference_golden(case):
    mfile, f, bcs, gfile, P = CASES[case]
    m = read_gmsh(path(mfile))
    rp, cols = O.sparsity(m.n_nodes, m.n_nodes, m.cells)
    vals, rhs = O.assemble_poisson(m.n_nodes, m.cells, m.coords, rp, cols, 0.0 if f is None else f)
    for g, v in bcs:
        O.dirichlet_penalty(m.group_nodes(g), v, P, rp, cols, vals, rhs)
    x = O.sequential_dense_solve(O.csr_to_dense(rp, cols, vals), rhs)
    gold = read_node_result_file(path(gfile))
    assert len(gold) == m.n_nodes
    nerr, mx = O.check_node_result({int(t): x[i] for i, t in enumerate(m.node_tags)}, gold, 1e-4)
    assert nerr == 0, f"{nerr} nodes outside the reference's 1e-4 gate"
    assert mx <= GOLDEN_TOL[case], f"max rel error {mx:.3e}"


def test_mesh_counts_match_survey():
    # circle_cut 101/166, sphere_cut 194/527, plancher 117/196,
    # L-shape 151/254, L-shape-3D 108/259, bar 80/122
    expect = {"circle_cut": (101, 166), "sphere_cut": (194, 527), "plancher": (117, 196), "L-shape": (151, 254),
              "L-shape-3D": (108, 259), "bar": (80, 122)}
    for name, (nn, nc) in expect.items():
        m = read_gmsh(path(name + ".msh"))
        assert (m.n_nodes, m.n_cells) == (nn, nc)


def test_element_known_answers():
    # reference tetrahedron: K = V * G G^T with V = 1/6, grads (-1,-1,-1), e1, e2, e3
    K, v = O.element_tet4(np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1]], dtype=float))
    G = np.array([[-1, -1, -1], [1, 0, 0], [0, 1, 0], [0, 0, 1]], dtype=float)
    assert abs(v - 1 / 6) < 1e-15
    assert np.allclose(K, G @ G.T / 6, atol=1e-15)
    # invariant to node order and orientation
    K2, _ = O.element_tet4(np.array([[0, 1, 0], [1, 0, 0], [0, 0, 0], [0, 0, 1]], dtype=float))
    perm = [2, 1, 0, 3]
    assert np.allclose(K2, K[np.ix_(perm, perm)], atol=1e-15)
    Kt, a = O.element_tri3(np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], dtype=float))
    assert abs(a - 0.5) < 1e-15
    assert np.allclose(Kt, np.array([[1, -0.5, -0.5], [-0.5, 0.5, 0], [-0.5, 0, 0.5]]), atol=1e-15)


def test_elasticity_element_rigid_modes():
    rng = np.random.default_rng(1)
    xyz = np.c_[rng.random((3, 2)), np.zeros(3)]
    K = O.element_elasticity_tri3(xyz, 1.2, 0.8)
    assert np.allclose(K, K.T, atol=1e-12 * np.abs(K).max())
    tx = np.tile([1.0, 0.0], 3)
    ty = np.tile([0.0, 1.0], 3)
    rot = np.ravel(np.c_[-xyz[:, 1], xyz[:, 0]])
    for mode in (tx, ty, rot):
        assert np.abs(K @ mode).max() < 1e-12 * np.abs(K).max()


def test_global_elasticity_rigid_modes_and_layouts():
    # the assembled block-2 matrix on the reference's bar mesh: symmetric, the
    # three planar rigid-body modes in its kernel, and the per-row (Hypre CSR)
    # layout a permutation of the per-block one
    m = read_gmsh(path("bar.msh"))
    rp, cols = O.sparsity(m.n_nodes, m.n_nodes, m.cells)
    v = O.assemble_elasticity_tri(m.n_nodes, m.cells, m.coords, rp, cols, 1.2e5, 1.6e5)
    n = m.n_nodes
    A = np.zeros((2 * n, 2 * n))
    for r in range(n):
        for k in range(rp[r], rp[r + 1]):
            A[2 * r:2 * r + 2, 2 * cols[k]:2 * cols[k] + 2] = v[4 * k:4 * k + 4].reshape(2, 2)
    scale = np.abs(A).max()
    assert np.abs(A - A.T).max() <= 1e-12 * scale
    x, y = m.coords[:, 0], m.coords[:, 1]
    for mode in (np.ravel(np.c_[np.ones(n), np.zeros(n)]), np.ravel(np.c_[np.zeros(n), np.ones(n)]),
                 np.ravel(np.c_[-y, x])):
        assert np.abs(A @ mode).max() <= 1e-10 * scale * max(1.0, np.abs(mode).max())
    w = O.blocks_to_row_order(rp, v)
    assert np.array_equal(np.sort(w), np.sort(v))
    r = 5
    ln = rp[r + 1] - rp[r]
    assert w[4 * rp[r] + 2 * ln] == v[4 * rp[r] + 2]  # (i=1, slot 0, j=0)


def test_sparsity_is_edge_graph():
    m = O.structured_mesh(3, 4)
    rp, cols = O.sparsity(m["n_local"], m["n_own"], m["cells"])
    # Kuhn interior node: 14 neighbours + diagonal
    assert np.diff(rp).max() == 15
    # rows sorted, diagonal present
    for r in range(m["n_own"]):
        seg = cols[rp[r]:rp[r + 1]]
        assert np.all(np.diff(seg) > 0) and r in seg
    # nnz = 2 E + N  (femutils/BSRFormat.h:397-399)
    edges = set()
    for c in m["cells"]:
        for a in range(4):
            for b in range(a + 1, 4):
                edges.add((min(c[a], c[b]), max(c[a], c[b])))
    assert rp[-1] == 2 * len(edges) + m["n_own"]


def test_structured_mesh_spec_slabs_cover_global_mesh():
    g = O.structured_mesh(3, 4, nz=6)
    seen = np.zeros(g["n_own"], dtype=int)
    for r in range(3):
        s = O.structured_mesh(3, 4, nz=6, nranks=3, rank=r)
        seen[s["local_to_global"][:s["n_own"]]] += 1
        assert np.array_equal(s["coords"], g["coords"][s["local_to_global"]])
    assert np.all(seen == 1)


def test_pcg_matches_direct():
    m = O.structured_mesh(3, 6)
    rp, cols = O.sparsity(m["n_local"], m["n_own"], m["cells"])
    vals, rhs = O.assemble_poisson(m["n_own"], m["cells"], m["coords"], rp, cols, 5.5)
    O.dirichlet_penalty(m["dirichlet"], 0.5, 1e30, rp, cols, vals, rhs)
    x, it, res, _ = O.pcg_jacobi(rp, cols, vals, rhs, rtol=1e-14)
    xd = np.linalg.solve(O.csr_to_dense(rp, cols, vals), rhs)
    assert np.abs(x - xd).max() / np.abs(xd).max() < 1e-10
    assert np.allclose(x[m["dirichlet"]], 0.5, atol=1e-14)


def test_pcg_dirichlet_driven_and_row_elimination():
    """No source term (Dirichlet data only) and row elimination (non-symmetric
    rows) both converge to the direct solution: the x0 lifting of the
    constraint rows (oracle.c::orc_pcg_jacobi, k_cg_x0)."""
    m = read_gmsh(path("plancher.msh"))
    rp, cols = O.sparsity(m.n_nodes, m.n_nodes, m.cells)
    vals, rhs = O.assemble_poisson(m.n_nodes, m.cells, m.coords, rp, cols, 0.0)
    for g, v in CASES["point_dirichlet_2D"][2]:
        O.dirichlet_penalty(m.group_nodes(g), v, 1e30, rp, cols, vals, rhs)
    x, it, res, _ = O.pcg_jacobi(rp, cols, vals, rhs, rtol=1e-14)
    xd = np.linalg.solve(O.csr_to_dense(rp, cols, vals), rhs)
    assert np.abs(x - xd).max() / np.abs(xd).max() < 1e-12
    m = read_gmsh(path("circle_cut.msh"))
    rp, cols = O.sparsity(m.n_nodes, m.n_nodes, m.cells)
    vals, rhs = O.assemble_poisson(m.n_nodes, m.cells, m.coords, rp, cols, 5.5)
    ids = m.group_nodes("horizontal")
    O.row_elimination(ids, 0.5, rp, cols, vals, rhs)
    x, it, res, _ = O.pcg_jacobi(rp, cols, vals, rhs, rtol=1e-14)
    xd = np.linalg.solve(O.csr_to_dense(rp, cols, vals), rhs)
    assert res <= 1e-14 and np.abs(x - xd).max() / np.abs(xd).max() < 1e-12
    assert np.all(x[ids] == 0.5)


# ---------------------------------------------------------------- Neumann / traction (K15)
from golden_cases import ELASTICITY_BAR, NEUMANN_CASES, lame  # noqa: E402


def oracle_neumann_system(m, f, dirichlet, neumann, P):
    rp, cols = O.sparsity(m.n_nodes, m.n_nodes, m.cells)
    vals, rhs = O.assemble_poisson(m.n_nodes, m.cells, m.coords, rp, cols, f)
    for g, v in neumann:
        faces = m.group_faces(g)
        O.neumann(m.dim, m.n_nodes, 1, O.NEUMANN_NORMAL, v, faces, m.face_cells(faces), m.cells, m.coords, rhs)
    for g, v in dirichlet:
        O.dirichlet_penalty(m.group_nodes(g), v, P, rp, cols, vals, rhs)
    return rp, cols, vals, rhs


@pytest.mark.parametrize("case", list(NEUMANN_CASES))
def test_oracle_neumann_reproduces_reference_golden(case):
    mfile, f, dirichlet, neumann, gfile, P = NEUMANN_CASES[case]
    m = read_gmsh(path(mfile))
    rp, cols, vals, rhs = oracle_neumann_system(m, f, dirichlet, neumann, P)
    x = O.sequential_dense_solve(O.csr_to_dense(rp, cols, vals), rhs)
    gold = read_node_result_file(path(gfile))
    nerr, mx = O.check_node_result({int(t): x[i] for i, t in enumerate(m.node_tags)}, gold, 1e-4)
    print(f"{case}: max rel error vs reference golden {mx:.3e}")
    assert nerr == 0 and mx <= 1e-8, f"max rel error {mx:.3e}"


def oracle_elasticity_bar():
    c = ELASTICITY_BAR
    m = read_gmsh(path(c["mesh"]))
    lam, mu2 = lame(c["E"], c["nu"])
    n = m.n_nodes
    rp, cols = O.sparsity(n, n, m.cells)
    v = O.assemble_elasticity_tri(n, m.cells, m.coords, rp, cols, lam, mu2)
    A = np.zeros((2 * n, 2 * n))
    for r in range(n):
        for k in range(rp[r], rp[r + 1]):
            A[2 * r:2 * r + 2, 2 * cols[k]:2 * cols[k] + 2] = v[4 * k:4 * k + 4].reshape(2, 2)
    b = np.zeros(2 * n)
    faces = m.group_faces(c["traction_group"])
    O.neumann(2, n, 2, O.NEUMANN_TRACTION, c["traction"], faces, None, m.cells, m.coords, b)
    clamp = m.group_nodes(c["clamp"])
    for i in range(2):
        d = 2 * clamp + i
        A[d, d] = c["penalty"]   # matrixSetValue(dof, dof, P) (modules/elasticity/FemModule.cc:300-306)
        b[d] = c["penalty"] * 0.0
    return m, A, b, rp, cols, v


def check_vector_golden(m, u, gfile, eps=1e-3, min_value=1e-16):
    gold = read_node_result_file(path(gfile))
    worst = 0.0
    nerr = 0
    for comp in range(2):
        g = {uid: val[comp] for uid, val in gold.items()}
        e, mx = O.check_node_result({int(t): u[2 * i + comp] for i, t in enumerate(m.node_tags)}, g, eps,
                                    min_value)
        nerr += e
        worst = max(worst, mx)
    return nerr, worst


def test_oracle_elasticity_traction_reproduces_reference_golden():
    """Pins the block-2 restatement (element matrix, traction RHS, penalty
    clamp) with the reference's own elasticity golden."""
    m, A, b, _, _, _ = oracle_elasticity_bar()
    u = O.sequential_dense_solve(A, b)
    nerr, mx = check_vector_golden(m, u, ELASTICITY_BAR["golden"])
    print(f"elasticity bar traction: max rel error vs reference golden {mx:.3e}")
    assert nerr == 0 and mx <= 1e-10, f"max rel error {mx:.3e}"
