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


def _tiny_box(n=2, seed=5):
    """Kuhn box of n^3 cubes (6 tets each), jittered interior nodes."""
    g = np.arange(n + 1)
    X, Y, Z = np.meshgrid(g, g, g, indexing="ij")
    coords = np.stack([X.ravel(), Y.ravel(), Z.ravel()], 1).astype(np.float64) / n
    rng = np.random.default_rng(seed)
    inner = np.all((coords > 0) & (coords < 1), axis=1)
    coords[inner] += (rng.random((inner.sum(), 3)) - 0.5) * 0.2 / n
    idx = lambda i, j, k: (i * (n + 1) + j) * (n + 1) + k  # noqa: E731
    cells = []
    for i in range(n):
        for j in range(n):
            for k in range(n):
                c = [idx(i + a, j + b, k + d) for a in (0, 1) for b in (0, 1) for d in (0, 1)]
                v0, v7 = c[0], c[7]
                for p in ((1, 3), (1, 5), (2, 3), (2, 6), (4, 5), (4, 6)):
                    cells.append([v0, c[p[0]], c[p[1]], v7])
    return np.asarray(cells, dtype=np.int32), coords


def test_time_constants_match_the_module():
    """c0 .. c10 of modules/elastodynamics/FemModule.cc:255-290: generalized
    alpha with alpm = alpf = 0 is Newmark-beta, damping terms vanish without
    etam / etak, and the undamped Newmark constants are the ones the C5 loop
    always used (rho / (beta dt^2), rho / (beta dt), rho (1 - 2 beta) / (2 beta))."""
    lam, mu, rho, dt = 1.7, 0.9, 2.5, 1e-2
    for etam, etak in ((0.0, 0.0), (0.3, 1e-3)):
        gn, bn, cn = O.elastodynamics_constants(lam, mu, rho, dt, etam, etak, scheme="newmark-beta")
        ga, ba, ca = O.elastodynamics_constants(lam, mu, rho, dt, etam, etak, 0.0, 0.0, scheme="generalized-alpha")
        assert (gn, bn) == (ga, ba) == (0.5, 0.25)
        assert np.allclose(cn, ca, rtol=1e-15, atol=0.0)
    _, _, c = O.elastodynamics_constants(lam, mu, rho, dt)
    assert c[0] == rho / (0.25 * dt * dt) and c[3] == rho / 0.25 / dt and c[4] == rho * (0.5 / 0.5)
    assert c[1] == lam and c[2] == 2 * mu and not any(c[5:])
    g, b, _ = O.elastodynamics_constants(lam, mu, rho, dt, alpm=0.2, alpf=0.4, scheme="generalized-alpha")
    assert abs(g - 0.7) < 1e-15 and abs(b - 0.25 * 1.2 ** 2) < 1e-15
    with pytest.raises(ValueError):
        O.elastodynamics_constants(lam, mu, rho, dt, scheme="hht")


def test_oracle_damped_loop():
    """The oracle's loop with Rayleigh damping: generalized alpha at
    alpm = alpf = 0 replays Newmark-beta bit for bit, and mass + stiffness
    damping take energy out of a free vibration (the undamped loop keeps
    it within 2 %)."""
    cells, coords = _tiny_box(2)
    n_nodes = coords.shape[0]
    fixed = np.nonzero(coords[:, 0] < 1e-12)[0]
    E, nu, rho, dt = 100.0, 0.3, 1.0, 2e-2
    args = (n_nodes, cells, coords, E, nu, rho, dt, 12, (0.0, 0.0, -1.0), fixed)
    Un, Vn, An = O.newmark_elastodynamics(*args, etam=0.2, etak=1e-3)
    Ua, Va, Aa = O.newmark_elastodynamics(*args, etam=0.2, etak=1e-3, scheme="generalized-alpha")
    assert np.array_equal(Un, Ua) and np.array_equal(Vn, Va) and np.array_equal(An, Aa)

    # a suddenly applied load: the undamped response oscillates about the
    # static deflection for ever, the damped one settles onto it
    lam = E * nu / ((1 + nu) * (1 - 2 * nu))
    mu2 = E / (1 + nu)
    rp, cols = O.sparsity(n_nodes, n_nodes, cells)
    n = 3 * n_nodes
    k_vals, f_rhs = O.assemble_elasticity_tet(n_nodes, cells, coords, rp, cols, lam, mu2, 0.0, (0.0, 0.0, -1.0))
    K = np.zeros((n, n))
    for r in range(n_nodes):
        for k in range(int(rp[r]), int(rp[r + 1])):
            K[3 * r:3 * r + 3, 3 * cols[k]:3 * cols[k] + 3] += k_vals[9 * k:9 * k + 9].reshape(3, 3)
    fx = (3 * fixed[:, None] + np.arange(3)).ravel()
    K[fx, :] = 0.0
    K[fx, fx] = 1.0
    f_rhs[fx] = 0.0
    Us = np.linalg.solve(K, f_rhs)
    dev = {}
    for tag, kw in (("undamped", {}), ("damped", dict(etam=4.0, etak=2e-3)),
                    ("alpha", dict(etam=4.0, etak=2e-3, alpm=0.2, alpf=0.4, scheme="generalized-alpha"))):
        dev[tag] = max(np.abs(O.newmark_elastodynamics(n_nodes, cells, coords, E, nu, rho, dt, s_, (0.0, 0.0, -1.0),
                                                       fixed, **kw)[0] - Us).max() for s_ in range(60, 72, 2))
    assert dev["damped"] < 0.3 * dev["undamped"], dev
    assert dev["alpha"] < 0.3 * dev["undamped"], dev
