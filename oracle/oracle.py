"""ORACLE — TEST INFRASTRUCTURE ONLY.

Python side of the CPU oracle: ctypes bindings to ``oracle/build/liboracle.so``
(the plain-C restatement of the reference, see oracle.c for the file:line each
function follows) plus numpy helpers:

* ``structured_mesh`` — the synthetic-input specification (jittered Kuhn
  tetrahedra / split squares, seeded counter-based hash).  The product path
  generates the same mesh on the GPU (``afem_mesh_create_structured``); the
  parity tests check the two agree bit for bit.
* ``sequential_dense_solve`` — the SequentialBasicDoFLinearSystem semantics of
  config C1 (dense N x N matrix, `femutils/DoFLinearSystem.cc:72-164`).
* ``check_node_result`` — the golden comparison of
  `femutils/FemUtils.cc:84-169` (relative epsilon, keyed by node unique id).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg import this module, as the checker or the timed CPU
baseline.  Parity status: pinned by the reference's golden result files
(tests/golden, replayed in tests/test_oracle_golden.py); the Arcane MatVec CG
stopping rule is external to the reference tree and therefore unpinned (the
goldens used here are all solved by the direct branch, N < 500).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "oracle.c")):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_element_tet4.argtypes = [_f64p, _f64p, ctypes.POINTER(ctypes.c_double)]
        L.orc_element_tri3.argtypes = [_f64p, _f64p, ctypes.POINTER(ctypes.c_double)]
        L.orc_element_elasticity_tri3.argtypes = [_f64p, ctypes.c_double, ctypes.c_double, _f64p]
        L.orc_element_elasticity_tet4.argtypes = [_f64p, ctypes.c_double, ctypes.c_double, ctypes.c_double, _f64p]
        L.orc_assemble_elasticity_tet.restype = ctypes.c_int64
        L.orc_assemble_elasticity_tet.argtypes = [ctypes.c_int64, ctypes.c_int64, _i32p, _f64p, _i64p, _i32p,
                                                  ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_void_p,
                                                  _f64p, ctypes.c_void_p]
        L.orc_sparsity.restype = ctypes.c_int64
        L.orc_sparsity.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, _i32p, _i64p,
                                   ctypes.c_void_p]
        L.orc_assemble_poisson.restype = ctypes.c_int64
        L.orc_assemble_poisson.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int, _i32p, _f64p, _i64p, _i32p,
                                           _f64p, ctypes.c_double, ctypes.c_void_p]
        L.orc_assemble_poisson_omp.restype = ctypes.c_int64
        L.orc_assemble_poisson_omp.argtypes = L.orc_assemble_poisson.argtypes
        L.orc_omp_threads.restype = ctypes.c_int
        L.orc_omp_threads.argtypes = [ctypes.c_int]
        L.orc_assemble_elasticity_tri.restype = ctypes.c_int64
        L.orc_assemble_elasticity_tri.argtypes = [ctypes.c_int64, ctypes.c_int64, _i32p, _f64p, _i64p, _i32p,
                                                  ctypes.c_double, ctypes.c_double, _f64p]
        L.orc_dirichlet_penalty.argtypes = [ctypes.c_int64, _i32p, ctypes.c_double, ctypes.c_double, _i64p, _i32p,
                                            _f64p, _f64p]
        L.orc_row_elimination.argtypes = [ctypes.c_int64, _i32p, ctypes.c_double, _i64p, _i32p, _f64p, _f64p]
        L.orc_spmv.argtypes = [ctypes.c_int64, _i64p, _i32p, _f64p, _f64p, _f64p]
        L.orc_pcg_jacobi.restype = ctypes.c_int
        L.orc_pcg_jacobi.argtypes = [ctypes.c_int64, _i64p, _i32p, _f64p, _f64p, _f64p, ctypes.c_double,
                                     ctypes.c_double, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_double)]
        L.orc_neumann.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int, _f64p, ctypes.c_int64,
                                  _i32p, ctypes.c_void_p, ctypes.c_int, _i32p, _f64p, _f64p]
        L.orc_eliminate.argtypes = [ctypes.c_int64, np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS"), _f64p,
                                    _i64p, _i32p, _f64p, _f64p]
        L.orc_pcg_jacobi_omp.restype = ctypes.c_int
        L.orc_pcg_jacobi_omp.argtypes = L.orc_pcg_jacobi.argtypes
        _lib = L
    return _lib


# --------------------------------------------------------------------------
# element matrices
# --------------------------------------------------------------------------
def element_tet4(xyz):
    xyz = np.ascontiguousarray(xyz, dtype=np.float64).reshape(4, 3)
    K = np.zeros(16)
    v = ctypes.c_double()
    lib().orc_element_tet4(xyz.ravel(), K, ctypes.byref(v))
    return K.reshape(4, 4), v.value


def element_tri3(xyz):
    xyz = np.ascontiguousarray(xyz, dtype=np.float64).reshape(3, 3)
    K = np.zeros(9)
    v = ctypes.c_double()
    lib().orc_element_tri3(xyz.ravel(), K, ctypes.byref(v))
    return K.reshape(3, 3), v.value


def element_elasticity_tri3(xyz, lam, mu2):
    xyz = np.ascontiguousarray(xyz, dtype=np.float64).reshape(3, 3)
    K = np.zeros(36)
    lib().orc_element_elasticity_tri3(xyz.ravel(), lam, mu2, K)
    return K.reshape(6, 6)


def element_elasticity_tet4(xyz, lam, mu2, c0=0.0):
    """12x12 block-3 elasticity (+ c0 * consistent mass) of one tetrahedron."""
    xyz = np.ascontiguousarray(xyz, dtype=np.float64).reshape(4, 3)
    K = np.zeros(144)
    lib().orc_element_elasticity_tet4(xyz.ravel(), lam, mu2, c0, K)
    return K.reshape(12, 12)


# --------------------------------------------------------------------------
# sparsity / assembly / BC / solve
# --------------------------------------------------------------------------
def sparsity(n_nodes, n_rows, cells):
    cells = np.ascontiguousarray(cells, dtype=np.int32)
    nv = cells.shape[1]
    row_ptr = np.zeros(n_rows + 1, dtype=np.int64)
    L = lib()
    nnz = L.orc_sparsity(n_nodes, n_rows, cells.shape[0], nv, cells.ravel(), row_ptr, None)
    cols = np.zeros(max(nnz, 1), dtype=np.int32)
    L.orc_sparsity(n_nodes, n_rows, cells.shape[0], nv, cells.ravel(), row_ptr,
                   cols.ctypes.data_as(ctypes.c_void_p))
    return row_ptr, cols[:nnz]


def assemble_poisson(n_rows, cells, coords, row_ptr, cols, f=0.0, with_rhs=True):
    """Matrix values (+ constant-source RHS) on a fixed structure."""
    cells = np.ascontiguousarray(cells, dtype=np.int32)
    coords = np.ascontiguousarray(coords, dtype=np.float64).reshape(-1, 3)
    vals = np.zeros(cols.shape[0], dtype=np.float64)
    rhs = np.zeros(n_rows, dtype=np.float64)
    missing = lib().orc_assemble_poisson(n_rows, cells.shape[0], cells.shape[1], cells.ravel(), coords.ravel(),
                                         row_ptr, cols, vals, f,
                                         rhs.ctypes.data_as(ctypes.c_void_p) if with_rhs else None)
    if missing:
        raise RuntimeError(f"{missing} (row,col) pairs missing from the structure")
    return vals, rhs


def omp_threads(n=0):
    """Set (n > 0) and return the OpenMP thread count of the multi-core oracle loop."""
    return lib().orc_omp_threads(n)


def assemble_poisson_omp(n_rows, cells, coords, row_ptr, cols, f=0.0):
    """assemble_poisson on all OpenMP threads (atomic adds, the reference's
    multi-core cell loop); bench.py's multi-core CPU baseline only."""
    cells = np.ascontiguousarray(cells, dtype=np.int32)
    coords = np.ascontiguousarray(coords, dtype=np.float64).reshape(-1, 3)
    vals = np.zeros(cols.shape[0], dtype=np.float64)
    rhs = np.zeros(n_rows, dtype=np.float64)
    missing = lib().orc_assemble_poisson_omp(n_rows, cells.shape[0], cells.shape[1], cells.ravel(), coords.ravel(),
                                             row_ptr, cols, vals, f, rhs.ctypes.data_as(ctypes.c_void_p))
    if missing:
        raise RuntimeError(f"{missing} (row,col) pairs missing from the structure")
    return vals, rhs


def assemble_elasticity_tri(n_rows, cells, coords, row_ptr, cols, lam, mu2):
    """Block-2 P1 elasticity values, ordered per block (block*4 + i*2 + j)."""
    cells = np.ascontiguousarray(cells, dtype=np.int32)
    coords = np.ascontiguousarray(coords, dtype=np.float64).reshape(-1, 3)
    vals = np.zeros(4 * cols.shape[0], dtype=np.float64)
    missing = lib().orc_assemble_elasticity_tri(n_rows, cells.shape[0], cells.ravel(), coords.ravel(), row_ptr, cols,
                                                lam, mu2, vals)
    if missing:
        raise RuntimeError(f"{missing} (row,col) blocks missing from the structure")
    return vals


def assemble_elasticity_tet(n_rows, cells, coords, row_ptr, cols, lam, mu2, c0=0.0, f=None):
    """Block-3 P1 elasticity (+ c0 mass) values ordered per block
    (block*9 + i*3 + j) and the body-force RHS (3 per owned node)."""
    cells = np.ascontiguousarray(cells, dtype=np.int32)
    coords = np.ascontiguousarray(coords, dtype=np.float64).reshape(-1, 3)
    vals = np.zeros(9 * cols.shape[0], dtype=np.float64)
    rhs = np.zeros(3 * n_rows, dtype=np.float64)
    fa = None if f is None else np.ascontiguousarray(f, dtype=np.float64)
    missing = lib().orc_assemble_elasticity_tet(n_rows, cells.shape[0], cells.ravel(), coords.ravel(), row_ptr, cols,
                                                lam, mu2, c0, None if fa is None else fa.ctypes.data_as(ctypes.c_void_p),
                                                vals, None if fa is None else rhs.ctypes.data_as(ctypes.c_void_p))
    if missing:
        raise RuntimeError(f"{missing} (row,col) blocks missing from the structure")
    return vals, rhs


def blocks_to_row_order_k(row_ptr, vals, k):
    """Per-block k x k values -> the per-scalar-row (CSR / Hypre) layout
    rb*k^2 + i*k*len + k*slot + j."""
    out = np.empty_like(vals)
    kk = k * k
    for r in range(row_ptr.shape[0] - 1):
        rb, re = int(row_ptr[r]), int(row_ptr[r + 1])
        ln = re - rb
        blk = vals[kk * rb:kk * re].reshape(ln, k, k)
        out[kk * rb:kk * re] = blk.transpose(1, 0, 2).reshape(-1)
    return out


def blocks_to_row_order(row_ptr, vals4):
    """Per-block 2x2 values -> the per-scalar-row (CSR / Hypre) layout
    rb*4 + i*2*len + 2*slot + j (femutils/BSRFormat.h:877-887)."""
    out = np.empty_like(vals4)
    for r in range(row_ptr.shape[0] - 1):
        rb, re = int(row_ptr[r]), int(row_ptr[r + 1])
        ln = re - rb
        blk = vals4[4 * rb:4 * re].reshape(ln, 2, 2)
        out[4 * rb:4 * re] = blk.transpose(1, 0, 2).reshape(-1)
    return out


NEUMANN_VALUE, NEUMANN_NORMAL, NEUMANN_TRACTION = 0, 1, 2


def neumann(dim, n_own, k, mode, value, faces, face_cells, cells, coords, rhs):
    """Adds the Neumann / traction term of the boundary faces to rhs in place
    (oracle.c::orc_neumann)."""
    v = np.zeros(3)
    v[:len(np.atleast_1d(value))] = np.atleast_1d(value)
    faces = np.ascontiguousarray(faces, dtype=np.int32)
    fc = None if face_cells is None else np.ascontiguousarray(face_cells, dtype=np.int32)
    cells = np.ascontiguousarray(cells, dtype=np.int32)
    coords = np.ascontiguousarray(coords, dtype=np.float64).reshape(-1, 3)
    lib().orc_neumann(dim, n_own, k, mode, v, faces.shape[0], faces.ravel(),
                      None if fc is None else fc.ctypes.data_as(ctypes.c_void_p), cells.shape[1], cells.ravel(),
                      coords.ravel(), rhs)
    return rhs


def dirichlet_penalty(dofs, value, penalty, row_ptr, cols, vals, rhs):
    dofs = np.ascontiguousarray(dofs, dtype=np.int32)
    lib().orc_dirichlet_penalty(dofs.shape[0], dofs, value, penalty, row_ptr, cols, vals, rhs)


def row_elimination(dofs, value, row_ptr, cols, vals, rhs):
    dofs = np.ascontiguousarray(dofs, dtype=np.int32)
    lib().orc_row_elimination(dofs.shape[0], dofs, value, row_ptr, cols, vals, rhs)


def eliminate(info, value, row_ptr, cols, vals, rhs):
    """Aleph row / row+column elimination (oracle.c::orc_eliminate); info 1 =
    eliminateRow, 2 = eliminateRowColumn; arrays updated in place."""
    n = row_ptr.shape[0] - 1
    lib().orc_eliminate(n, np.ascontiguousarray(info, dtype=np.uint8), np.ascontiguousarray(value, dtype=np.float64),
                        row_ptr, cols, vals, rhs)


def spmv(row_ptr, cols, vals, x):
    n = row_ptr.shape[0] - 1
    y = np.zeros(n)
    lib().orc_spmv(n, row_ptr, cols, vals, np.ascontiguousarray(x, dtype=np.float64), y)
    return y


def pcg_jacobi(row_ptr, cols, vals, b, rtol=1e-12, atol=0.0, max_iter=10000, x0=None):
    n = row_ptr.shape[0] - 1
    x = np.zeros(n) if x0 is None else np.array(x0, dtype=np.float64)
    res = ctypes.c_double()
    rn = ctypes.c_double()
    it = lib().orc_pcg_jacobi(n, row_ptr, cols, vals, np.ascontiguousarray(b, dtype=np.float64), x, rtol, atol,
                              max_iter, ctypes.byref(res), ctypes.byref(rn))
    return x, it, res.value, rn.value


def pcg_jacobi_omp(row_ptr, cols, vals, b, rtol=1e-12, atol=0.0, max_iter=10000):
    """orc_pcg_jacobi on all the OpenMP threads (omp_threads); max_iter < 0: exactly
    -max_iter iterations."""
    n = row_ptr.shape[0] - 1
    x = np.zeros(n)
    res = ctypes.c_double()
    rn = ctypes.c_double()
    it = lib().orc_pcg_jacobi_omp(n, row_ptr, cols, vals, np.ascontiguousarray(b, dtype=np.float64), x, rtol, atol,
                                  max_iter, ctypes.byref(res), ctypes.byref(rn))
    return x, it, res.value, rn.value


def csr_to_dense(row_ptr, cols, vals, n_cols=None):
    n = row_ptr.shape[0] - 1
    m = n if n_cols is None else n_cols
    A = np.zeros((n, m))
    for r in range(n):
        s, e = row_ptr[r], row_ptr[r + 1]
        np.add.at(A[r], cols[s:e], vals[s:e])  # duplicate (r, c) entries add up
    return A


def sequential_dense_solve(A, b, epsilon=1e-15):
    """SequentialDoFLinearSystemImpl::solve (femutils/DoFLinearSystem.cc:106-164):
    dense -> CSR dropping exact zeros (femutils/FemUtils.cc:35-76), direct
    solver when N < 500, else diagonal-preconditioned CG with epsilon."""
    n = A.shape[0]
    if n < 500:
        return np.linalg.solve(A, b)
    mask = A != 0.0
    row_ptr = np.concatenate([[0], np.cumsum(mask.sum(axis=1))]).astype(np.int64)
    r, c = np.nonzero(mask)
    x, _, _, _ = pcg_jacobi(row_ptr, c.astype(np.int32), A[r, c].copy(), b, rtol=epsilon, max_iter=20 * n)
    return x


# --------------------------------------------------------------------------
# synthetic structured meshes (the input specification shared with the GPU
# generator; see DESIGN.md "Synthetic inputs")
# --------------------------------------------------------------------------
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
KUHN_PERMS = ((0, 1, 2), (0, 2, 1), (1, 0, 2), (1, 2, 0), (2, 0, 1), (2, 1, 0))


def hash_u01(seed: int, idx: np.ndarray) -> np.ndarray:
    """splitmix64(seed + (idx+1)*golden) -> double in [0,1) with 53 bits."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (idx.astype(np.uint64) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def slab_range(nz: int, nranks: int, rank: int):
    """Owned node layers [k0, k1) of `rank` in a z-slab split of nz+1 layers."""
    nl = nz + 1
    return rank * nl // nranks, (rank + 1) * nl // nranks


def structured_mesh(dim, n, nz=None, jitter=0.2, seed=20250220, nranks=1, rank=0):
    """Jittered structured mesh of the unit square (2D: 2 triangles per square)
    or the box [0,1]^2 x [0, nz/n] (3D: 6 Kuhn tetrahedra per cube), cut into
    `nranks` z-slabs (y-slabs in 2D).  Returns dict with coords [n_local,3],
    cells [n_cells,nv] (local ids: owned nodes first, then ghost nodes),
    n_own, local_to_global, and dirichlet (local ids of owned nodes on the
    z=0 (2D: y=0) face)."""
    nz = n if nz is None else nz
    h = 1.0 / n
    amp = jitter * h
    nx = ny = n
    if dim == 3:
        L = (nx + 1) * (ny + 1)
        nlayers = nz + 1
    else:
        L = nx + 1
        nlayers = ny + 1
        nz = ny
    k0, k1 = slab_range(nz, nranks, rank)
    layers = list(range(k0, k1))
    ghost = []
    if k0 > 0:
        ghost.append(k0 - 1)
    if k1 < nlayers:
        ghost.append(k1)
    all_layers = layers + ghost
    # global ids of local nodes
    inplane = np.arange(L, dtype=np.int64)
    l2g = np.concatenate([inplane + k * L for k in all_layers]) if all_layers else np.zeros(0, np.int64)
    g2l_layer = {k: idx for idx, k in enumerate(all_layers)}
    g = l2g
    if dim == 3:
        i = g % (nx + 1)
        j = (g // (nx + 1)) % (ny + 1)
        k = g // L
        comps = [i, j, k]
    else:
        i = g % (nx + 1)
        j = g // (nx + 1)
        comps = [i, j]
    coords = np.zeros((g.shape[0], 3))
    for c, ic in enumerate(comps):
        u = hash_u01(seed, g * 3 + c)
        coords[:, c] = ic.astype(np.float64) * h + (u - 0.5) * amp
    n_own = len(layers) * L

    def lid(gid):
        layer = gid // L
        pos = gid % L
        return np.array([g2l_layer[int(x)] for x in np.atleast_1d(layer)]).reshape(np.shape(gid)) * L + pos

    # cells touching owned nodes: cell layers [max(k0-1,0), min(k1, nz))
    c_lo, c_hi = max(k0 - 1, 0), min(k1, nz)
    if dim == 3:
        ci, cj, ck = np.meshgrid(np.arange(nx), np.arange(ny), np.arange(c_lo, c_hi), indexing="ij")
        ci, cj, ck = (a.transpose(2, 1, 0).ravel() for a in (ci, cj, ck))  # lexicographic: i fastest
        e = np.eye(3, dtype=np.int64)
        tets = []
        for perm in KUHN_PERMS:
            v0 = np.stack([ci, cj, ck], 1)
            v1 = v0 + e[perm[0]]
            v2 = v1 + e[perm[1]]
            v3 = v0 + 1
            tets.append(np.stack([v0, v1, v2, v3], 1))  # [ncube, 4, 3]
        T = np.stack(tets, 1).reshape(-1, 4, 3)  # cube-major, 6 tets per cube
        gid = T[..., 0] + (nx + 1) * (T[..., 1] + (ny + 1) * T[..., 2])
    else:
        ci, cj = np.meshgrid(np.arange(nx), np.arange(c_lo, c_hi), indexing="xy")
        ci, cj = ci.ravel(), cj.ravel()
        v00 = ci + (nx + 1) * cj
        v10 = v00 + 1
        v01 = v00 + (nx + 1)
        v11 = v01 + 1
        gid = np.stack([np.stack([v00, v10, v11], 1), np.stack([v00, v11, v01], 1)], 1).reshape(-1, 3)
    layer = gid // L
    pos = gid % L
    lut = np.full(nlayers, -1, dtype=np.int64)
    for kk, idx in g2l_layer.items():
        lut[kk] = idx
    cells = (lut[layer] * L + pos).astype(np.int32)
    dirichlet = np.arange(L, dtype=np.int32) if k0 == 0 else np.zeros(0, np.int32)
    return dict(coords=coords, cells=cells, n_own=n_own, n_local=g.shape[0], local_to_global=l2g,
                dirichlet=dirichlet, dim=dim)


# --------------------------------------------------------------------------
# golden comparison (femutils/FemUtils.cc:84-169)
# --------------------------------------------------------------------------
def is_nearly_equal(ref, v, eps):
    d = abs(ref - v)
    if d == 0.0:
        return True
    return d < (abs(ref) + abs(v)) * eps


def check_node_result(values_by_uid: dict, golden: dict, eps: float, min_value: float = 0.0):
    """Returns (nb_error, max_rel) with Arcane's comparison semantics."""
    nb_error = 0
    max_rel = 0.0
    for uid, v in values_by_uid.items():
        if uid not in golden:
            continue
        ref = golden[uid]
        if abs(ref) < min_value and abs(v) < min_value:
            continue
        denom = max(abs(ref), abs(v), 1e-300)
        max_rel = max(max_rel, abs(ref - v) / denom)
        if not is_nearly_equal(ref, v, eps):
            nb_error += 1
    return nb_error, max_rel


def elastodynamics_constants(lam, mu, rho, dt, etam=0.0, etak=0.0, alpm=0.0, alpf=0.0, scheme="newmark-beta"):
    """gamma, beta and c0 .. c10 of modules/elastodynamics/FemModule.cc:255-290
    (Newmark-beta :256-270, generalized-alpha :275-290; Rayleigh damping
    etam, etak)."""
    if scheme == "generalized-alpha":
        gamma = 0.5 + alpf - alpm
        beta = (1.0 / 4.0) * (gamma + 0.5) * (gamma + 0.5)
        c = [rho * (1. - alpm) / (beta * dt * dt) + etam * rho * gamma * (1 - alpf) / beta / dt,
             lam * (1. - alpf) + lam * etak * gamma * (1. - alpf) / beta / dt,
             2. * mu * (1. - alpf) + 2. * mu * etak * gamma * (1. - alpf) / beta / dt,
             rho * (1. - alpm) / beta / dt - etam * rho * (1 - gamma * (1 - alpf) / beta),
             rho * ((1. - alpm) * (1. - 2. * beta) / 2. / beta - alpm - etam * dt * (1. - alpf) * (1. - gamma / 2 / beta)),
             lam * alpf - lam * etak * gamma * (1. - alpf) / beta / dt,
             2 * mu * alpf - 2. * mu * etak * gamma * (1. - alpf) / beta / dt,
             etak * lam * (gamma * (1. - alpf) / beta - 1),
             etak * lam * dt * (1. - alpf) * ((1. - 2 * beta) / 2. / beta - (1. - gamma)),
             etak * 2 * mu * (gamma * (1. - alpf) / beta - 1),
             etak * 2 * mu * dt * (1. - alpf) * ((1. - 2 * beta) / 2. / beta - (1. - gamma))]
    elif scheme == "newmark-beta":
        gamma = 0.5
        beta = (1. / 4.) * (gamma + 0.5) * (gamma + 0.5)
        c = [rho / (beta * dt * dt) + etam * rho * gamma / beta / dt,
             lam + lam * etak * gamma / beta / dt,
             2. * mu + 2. * mu * etak * gamma / beta / dt,
             rho / beta / dt - etam * rho * (1 - gamma / beta),
             rho * ((1. - 2. * beta) / 2. / beta - etam * dt * (1. - gamma / 2 / beta)),
             -lam * etak * gamma / beta / dt,
             -2. * mu * etak * gamma / beta / dt,
             etak * lam * (gamma / beta - 1),
             etak * lam * dt * ((1. - 2 * beta) / 2. / beta - (1. - gamma)),
             etak * 2 * mu * (gamma / beta - 1),
             etak * 2 * mu * dt * ((1. - 2 * beta) / 2. / beta - (1. - gamma))]
    else:
        raise ValueError("Only Newmark-beta | Generalized-alpha are supported for time-discretization")
    return gamma, beta, c


def newmark_elastodynamics(n_nodes, cells, coords, E, nu, rho, dt, n_steps, body_force, fixed_nodes, penalty=1e30,
                           etam=0.0, etak=0.0, alpm=0.0, alpf=0.0, scheme="newmark-beta"):
    """CPU restatement of the 3D elastodynamics time loop (per-step
    re-assembly; modules/elastodynamics/FemModule.cc:255-290 coefficients,
    LHS c0 M + K(lambda -> c1, 2 mu -> c2) (:1130-1340), :842-862 RHS
    M (c0 U + c3 V + c4 A) - K(c5, c6) U + K(c7, c9) V + K(c8, c10) A + body
    force, :429-455 update) on the oracle's block-3 assembly, penalty Dirichlet
    (diagonal set to P, rhs = P*0) and a dense direct solve.  Returns U, V, A
    (3 per node) after n_steps."""
    lam = E * nu / ((1 + nu) * (1 - 2 * nu))
    mu = E / (2 * (1 + nu))
    gamma, beta, c = elastodynamics_constants(lam, mu, rho, dt, etam, etak, alpm, alpf, scheme)
    c0, c3, c4 = c[0], c[3], c[4]
    rp, cols = sparsity(n_nodes, n_nodes, cells)
    m_vals, _ = assemble_elasticity_tet(n_nodes, cells, coords, rp, cols, 0.0, 0.0, 1.0)
    n = 3 * n_nodes

    def dense(vals):
        A = np.zeros((n, n))
        for r in range(n_nodes):
            for k in range(int(rp[r]), int(rp[r + 1])):
                A[3 * r:3 * r + 3, 3 * cols[k]:3 * cols[k] + 3] += vals[9 * k:9 * k + 9].reshape(3, 3)
        return A

    M = dense(m_vals)
    # K(lambda', 2 mu') of the RHS terms: div-div and strain parts, linear in the two moduli
    KL = dense(assemble_elasticity_tet(n_nodes, cells, coords, rp, cols, 1.0, 0.0, 0.0)[0])
    KM = dense(assemble_elasticity_tet(n_nodes, cells, coords, rp, cols, 0.0, 1.0, 0.0)[0])
    fixed = (3 * np.asarray(fixed_nodes)[:, None] + np.arange(3)[None, :]).ravel()
    U, V, A = np.zeros(n), np.zeros(n), np.zeros(n)
    for _ in range(n_steps):
        k_vals, f_rhs = assemble_elasticity_tet(n_nodes, cells, coords, rp, cols, c[1], c[2], c0, body_force)
        L = dense(k_vals)
        b = f_rhs + M @ (c0 * U + c3 * V + c4 * A)
        b += KL @ (-c[5] * U + c[7] * V + c[8] * A) + KM @ (-c[6] * U + c[9] * V + c[10] * A)
        L[fixed, fixed] = penalty
        b[fixed] = penalty * 0.0
        Un = np.linalg.solve(L, b)
        an = (Un - U - dt * V) / beta / (dt * dt) - (1.0 - 2.0 * beta) / 2.0 / beta * A
        V = V + dt * ((1.0 - gamma) * A + gamma * an)
        A = an
        U = Un
    return U, V, A


# --------------------------------------------------------------------------
# passmo: the reference's 3D elastodynamics (modules/passmo), P1 tetrahedra
# --------------------------------------------------------------------------
# 4-point Gauss rule of order 2 on the reference tetrahedron
# (femutils/GaussQuadrature.h:202, 209-241; ArcaneFemFunctions.h:2359-2396,
# 2503-2508, 2583-2587): points (a2,a2,a2), (a2,a2,b2), (a2,b2,a2), (b2,a2,a2)
# in (x,y,z) = xtet/ytet/ztet[1][rank], weight 1/24 each.
_PM_A2 = (5.0 - np.sqrt(5.0)) / 20.0
_PM_B2 = (5.0 + 3.0 * np.sqrt(5.0)) / 20.0
_PM_GAUSS = [(_PM_A2, _PM_A2, _PM_A2), (_PM_A2, _PM_A2, _PM_B2), (_PM_A2, _PM_B2, _PM_A2), (_PM_B2, _PM_A2, _PM_A2)]
_PM_WEIGHT = 1.0 / 24.0
# Tetra4 reference shape functions (ArcaneFemFunctions.h:1973-2004)
_PM_DPHI = np.array([[-1.0, -1.0, -1.0], [1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [0.0, 0.0, 1.0]])


def _pm_phi(r):
    x, y, z = r
    return np.array([1.0 - x - y - z, x, y, z])


def passmo_element_tet4(xyz, lam, mu, rho):
    """Per-Gauss-point element stiffness and mass of a P1 tetrahedron exactly
    as modules/passmo/ElastodynamicModule.cc computes them: Jacobian matrix
    jac[i][j] = sum_n dPhi_n[i] x_n[j] and its determinant (_initGaussStep,
    :414-465), B = jac^-1 dPhi (_computeK :1450-1478), Voigt B_ii / B_jj rows
    and kij = wt (B_ii^T D B_jj), D = [[a,l,l],[l,a,l],[l,l,a]] + mu on the
    shear terms, wt = w_g det (:1483-1573); Me(ii,jj) = wt rho Phi_i Phi_j on
    equal components (_computeElemMass :1390-1420).  Returns the two lists of
    the 4 Gauss points' 12x12 matrices (DoF 3 node + component)."""
    X = np.asarray(xyz, dtype=np.float64).reshape(4, 3)
    jac = _PM_DPHI.T @ X  # jac[i][j] = sum_n dPhi_n[i] * x_n[j]
    det = np.linalg.det(jac)
    ijac = np.linalg.inv(jac)
    a = lam + 2.0 * mu
    Ks, Ms = [], []
    for g in _PM_GAUSS:
        wt = _PM_WEIGHT * det
        B = ijac @ _PM_DPHI.T  # [3, 4]: B(i, inod) = sum_j ijac[i][j] dPhi_inod[j]
        V = np.zeros((12, 6))  # Voigt row of DoF 3 inod + l: (xx, yy, zz, xy, xz, yz)
        for n in range(4):
            bx, by, bz = B[:, n]
            V[3 * n + 0] = (bx, 0.0, 0.0, by, bz, 0.0)
            V[3 * n + 1] = (0.0, by, 0.0, bx, 0.0, bz)
            V[3 * n + 2] = (0.0, 0.0, bz, 0.0, bx, by)
        D = np.array([[a, lam, lam, 0, 0, 0], [lam, a, lam, 0, 0, 0], [lam, lam, a, 0, 0, 0],
                      [0, 0, 0, mu, 0, 0], [0, 0, 0, 0, mu, 0], [0, 0, 0, 0, 0, mu]], dtype=np.float64)
        Ks.append(wt * (V @ D @ V.T))
        phi = _pm_phi(g)
        M = np.zeros((12, 12))
        for i in range(4):
            for j in range(4):
                for comp in range(3):
                    M[3 * i + comp, 3 * j + comp] = wt * rho * phi[i] * phi[j]
        Ms.append(M)
    return Ks, Ms


def passmo_time_steps(start, final, dt):
    """The time steps modules/passmo/ElastodynamicModule.cc::compute (:469-536)
    takes: Arcane advances globalTime by deltat before each compute; a step
    whose t + dt overshoots the final time shortens the NEXT step to
    final - t (:525-530); the step that reaches t >= final checks the result
    file and stops the loop.  Returns the list of dt of the executed steps."""
    t, dts = start, []
    while True:
        t = t + dt
        dts.append(dt)
        if t < final:
            if t + dt > final:
                dt = final - t
        else:
            return dts


def passmo_newmark(cells, coords, lam, mu, rho, dts, imposed, penalty=1.0e64, beta=0.25, gamma=0.5):
    """CPU restatement of the passmo 3D Newmark loop (P1 tetrahedra, Penalty
    Dirichlet, no gravity / traction / paraxial terms, alfam = alfaf = 0):
    per step the LHS sum over the cell's Gauss points of cm Me + Ke with
    cm = 1/beta/dt^2 (_assembleLinearLHS :1709-1793, matrixAddValue of every
    (node1 own, node2) pair); the RHS of non-imposed DoFs sum_g Me(ii,jj)
    cm u_pred_j with u_pred = d + dt v + dt^2 (1/2 - beta) a (:1799-1915);
    imposed DoFs matrixSetValue(diag, penalty) (Aleph: the set overrides the
    adds) and rhs = u penalty (:1923-1939); a direct solve (the reference's
    solver converges to ~1e-9 on the golden); the imposed displacements
    re-applied after the solve (_doSolve :2343-2371); the Newmark update
    a = (d1 - u_pred)/beta/dt^2, v = v + dt (1-gamma) a_n + dt gamma a
    (_updateNewmark :555-591).  `imposed`: dict DoF -> value (DoF = 3 node +
    component).  Returns U, V, A after the steps."""
    cells = np.asarray(cells)
    coords = np.asarray(coords, dtype=np.float64).reshape(-1, 3)
    n = 3 * coords.shape[0]
    elems = [passmo_element_tet4(coords[c], lam, mu, rho) for c in cells]
    dofs = [(3 * np.asarray(c)[:, None] + np.arange(3)[None, :]).ravel() for c in cells]
    imp = np.array(sorted(imposed), dtype=np.int64)
    val = np.array([imposed[d] for d in imp], dtype=np.float64)
    U, V, A = np.zeros(n), np.zeros(n), np.zeros(n)
    free = np.ones(n, dtype=bool)
    free[imp] = False
    for dt in dts:
        dt2 = dt * dt
        cm = 1.0 / beta / dt2
        L = np.zeros((n, n))
        b = np.zeros(n)
        upred = U + dt * V + dt2 * (0.5 - beta) * A
        for d, (Ks, Ms) in zip(dofs, elems):
            for Ke, Me in zip(Ks, Ms):
                L[np.ix_(d, d)] += cm * Me + Ke
                b[d] += np.where(free[d], Me @ (cm * upred[d]), 0.0)
        L[imp, imp] = penalty
        b[imp] = val * penalty
        d1 = np.linalg.solve(L, b)
        d1[imp] = val
        an = (d1 - upred) / beta / dt2
        V = V + dt * (1.0 - gamma) * A + dt * gamma * an
        A, U = an, d1
    return U, V, A


# --------------------------------------------------------------------------
# extended-precision reference of the P1 Laplacian values (test infrastructure)
# --------------------------------------------------------------------------
def assemble_poisson_extended(n_rows, cells, coords, row_ptr, cols):
    """The assembled P1 Laplacian values in x87 extended precision (numpy
    longdouble, 64-bit mantissa) from edge vectors: K_ab = (c_a . c_b) /
    (6 |det|) (tets; triangles (c_a . c_b) / (2 |A2|)), c the cofactors.  The
    same bilinear form as the reference's element routines, computed ~2^11
    times more precisely than any double restatement, so that the per-entry
    error of a double implementation can be measured against it (entries that
    nearly cancel are ill-conditioned in every double formula).  Returns
    (values, magnitude) with magnitude = sum over the entry's terms of
    |c_a||c_b| / (6|det|) (the entry's condition scale)."""
    ld = np.longdouble
    cells = np.asarray(cells, dtype=np.int64)
    X = np.asarray(coords, dtype=np.float64).reshape(-1, 3).astype(ld)
    nv = cells.shape[1]
    P = X[cells]  # [nc, nv, 3]
    if nv == 4:
        e1, e2, e3 = P[:, 1] - P[:, 0], P[:, 2] - P[:, 0], P[:, 3] - P[:, 0]
        c1, c2, c3 = np.cross(e2, e3), np.cross(e3, e1), np.cross(e1, e2)
        c0 = -(c1 + c2 + c3)
        det = np.abs(np.sum(e1 * c1, axis=1))
        C = np.stack([c0, c1, c2, c3], 1)
        scale = 1 / (6 * det)
    else:
        e1, e2 = P[:, 1] - P[:, 0], P[:, 2] - P[:, 0]
        c1 = np.stack([e2[:, 1], -e2[:, 0]], 1)
        c2 = np.stack([-e1[:, 1], e1[:, 0]], 1)
        c0 = -(c1 + c2)
        det = np.abs(e1[:, 0] * e2[:, 1] - e2[:, 0] * e1[:, 1])
        C = np.stack([c0, c1, c2], 1)
        scale = 1 / (2 * det)
    K = np.einsum("cad,cbd->cab", C, C) * scale[:, None, None]
    M = np.einsum("cad,cbd->cab", np.abs(C), np.abs(C)) * scale[:, None, None]
    rows_idx = np.repeat(cells[:, :, None], nv, axis=2).ravel()
    cols_idx = np.repeat(cells[:, None, :], nv, axis=1).ravel()
    own = rows_idx < n_rows
    n_cols = int(max(cols.max() if cols.size else 0, cells.max() if cells.size else 0)) + 1
    keys = rows_idx[own] * n_cols + cols_idx[own]
    rid = np.repeat(np.arange(n_rows, dtype=np.int64), np.diff(row_ptr))
    ckeys = rid * n_cols + cols.astype(np.int64)
    pos = np.searchsorted(ckeys, keys)
    vals = np.zeros(cols.shape[0], dtype=ld)
    mag = np.zeros(cols.shape[0], dtype=ld)
    np.add.at(vals, pos, K.ravel()[own])
    np.add.at(mag, pos, M.ravel()[own])
    return vals, mag
