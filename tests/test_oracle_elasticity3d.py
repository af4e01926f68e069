"""Known answers pinning the oracle's block-3 tetrahedral elasticity
restatement, beside the reference pin of tests/test_oracle_passmo.py (the
passmo module assembles 3D P1 elasticity + mass on the CPU,
modules/passmo/ElastodynamicModule.cc:1389-1793, and its bar3d-tetra golden
fixes the element and the Newmark loop; SURVEY.md §8c had missed it): symmetry, exactly six
rigid-body zero modes, the patch test (exact strain energy of a uniform
strain), consistent mass summing to the volume, and reduction to the
reference's 2D TRIA3 element for plane-strain prisms is not attempted (the
3D and 2D meshes differ); instead the 2D restatement is pinned by the
reference elasticity golden (tests/test_oracle_golden.py)."""
import numpy as np
import pytest

from oracle import oracle as O


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_tet_element_known_answers(seed):
    rng = np.random.default_rng(seed)
    x = rng.random((4, 3))
    lam, mu2 = 1.3, 0.7
    K = O.element_elasticity_tet4(x, lam, mu2)
    scale = np.abs(K).max()
    assert np.abs(K - K.T).max() <= 1e-15 * scale
    modes = []
    for d in range(3):
        u = np.zeros(12)
        u[d::3] = 1.0
        modes.append(u)
    for ax in range(3):
        w = np.zeros(3)
        w[ax] = 1.0
        modes.append(np.concatenate([np.cross(w, p) for p in x]))
    for u in modes:
        assert np.abs(K @ u).max() <= 1e-13 * scale
    ev = np.linalg.eigvalsh(K)
    assert np.sum(np.abs(ev) < 1e-10 * ev.max()) == 6
    # patch test: u = G x with symmetric strain eps = sym(G)
    G = rng.random((3, 3))
    eps = (G + G.T) / 2
    u = np.concatenate([G @ p for p in x])
    vol = abs(np.linalg.det(np.array([x[1] - x[0], x[2] - x[0], x[3] - x[0]]))) / 6
    energy = vol * (lam * np.trace(eps) ** 2 + mu2 * np.sum(eps * eps))
    assert abs(u @ K @ u - energy) <= 1e-12 * energy
    M = O.element_elasticity_tet4(x, 0.0, 0.0, 1.0)
    assert abs(M.sum() / 3 - vol) <= 1e-14
    assert np.allclose(M[0::3, 0::3], vol / 20 * (np.ones((4, 4)) + np.eye(4)), rtol=1e-14, atol=0)


def test_global_tet_assembly_rigid_modes():
    m = O.structured_mesh(3, 3)
    cells, coords, n = m["cells"], m["coords"], m["n_own"]
    rp, cols = O.sparsity(m["n_local"], n, cells)
    vals, rhs = O.assemble_elasticity_tet(n, cells, coords, rp, cols, 2.0, 1.5, 0.0, (1.0, 2.0, 3.0))
    rid = np.repeat(np.arange(n), np.diff(rp))
    blk = vals.reshape(-1, 3, 3)
    for d in range(3):
        u = np.zeros((n, 3))
        u[:, d] = 1.0
        r = np.zeros((n, 3))
        np.add.at(r, rid, np.einsum("kij,kj->ki", blk, u[cols]))
        assert np.abs(r).max() <= 1e-12 * np.abs(vals).max()
    # body force: total load = f * volume of the (jittered) box
    x = coords[cells]
    vol = np.abs(np.linalg.det(np.stack([x[:, 1] - x[:, 0], x[:, 2] - x[:, 0], x[:, 3] - x[:, 0]], 1))).sum() / 6
    assert np.allclose(rhs.reshape(-1, 3).sum(0), np.array([1.0, 2.0, 3.0]) * vol, rtol=1e-12)
