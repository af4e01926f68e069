"""Host-side mirror of the reference's plugin surface over the C ABI.

Names and argument meaning follow toutane/arcanefem (femutils/):

* ``DoFLinearSystem``        femutils/DoFLinearSystem.h:126-286 (facade; owns the impl)
* ``HipDoFLinearSystemFactory`` femutils/IDoFLinearSystemFactory.h:34-44
* ``BSRFormat``              femutils/BSRFormat.h:353-1140
* ``Mesh``                   the subset of Arcane's IMesh the path reads
                             (cell->node connectivity, VariableNodeReal3 coordinates,
                             isOwn()) plus the synthetic structured generator

Device arrays are raw device addresses (ints) owned by the handles; ``*_host``
helpers copy them to numpy.  Errors are raised as ``AfemError`` (the
reference raises ARCANE_FATAL / NotImplementedException / ArgumentException).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _capi as C
from ._capi import AfemError, call

__all__ = ["AfemError", "Context", "Mesh", "BSRFormat", "DoFLinearSystem", "HipDoFLinearSystemFactory",
           "applyNeumannToRhs", "device_count", "set_variant", "structured_halo_plan"]


def _ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


def _rhs_mode(mode: str) -> int:
    if mode not in ("add", "set"):
        raise ValueError(f"rhs_mode must be 'add' or 'set', got {mode!r}")
    return C.AFEM_RHS_ADD if mode == "add" else C.AFEM_RHS_SET


NEUMANN_MODES = {"value": C.AFEM_NEUMANN_VALUE, "normal": C.AFEM_NEUMANN_NORMAL, "traction": C.AFEM_NEUMANN_TRACTION}


def applyNeumannToRhs(mesh: "Mesh", rhs_dptr: int, faces, value, mode: str = "normal", nb_dof: int = 1,
                      face_cells=None):
    """BoundaryConditions{2D,3D}::applyNeumannToRhs (femutils/ArcaneFemFunctionsGpu.h:612-766)
    and the elasticity traction term (modules/elasticity/FemModule.cc:244-273):
    adds the boundary-face term of `faces` (host int32 [n_faces, dim] local
    node ids) to the device RHS.  mode "value": scalar g; "normal": (v . n)
    with the outward normal (oriented by `face_cells`); "traction": vector t,
    one component per DoF."""
    faces = np.ascontiguousarray(faces, dtype=np.int32).reshape(-1, mesh.dim)
    v = np.zeros(3)
    vv = np.atleast_1d(np.asarray(value, dtype=np.float64))
    v[:vv.shape[0]] = vv
    fc = None if face_cells is None else np.ascontiguousarray(face_cells, dtype=np.int32)
    call("afem_apply_neumann", mesh.h, nb_dof, NEUMANN_MODES[mode], _ptr(v), faces.shape[0], _ptr(faces),
         None if fc is None else _ptr(fc), C.AFEM_MEM_HOST, ctypes.c_void_p(rhs_dptr))


def set_variant(name: str, value=None):
    """afem_set_variant: select a kernel variant (diagnostics / A-B runs;
    include/arcanefem_amd.h lists the knobs); None returns to the default."""
    call("afem_set_variant", name.encode(), None if value is None else str(value).encode())


def device_count() -> int:
    c = ctypes.c_int(0)
    call("afem_device_count", ctypes.byref(c))
    return c.value


class Context:
    """A device and the HIP stream every handle built on it enqueues to."""

    def __init__(self, device: int = 0, stream: int | None = None):
        h = ctypes.c_void_p()
        call("afem_ctx_create", device, ctypes.c_void_p(stream) if stream else None, ctypes.byref(h))
        self.h = h
        self.device = device

    def synchronize(self):
        call("afem_ctx_synchronize", self.h)

    def timer_start(self):
        call("afem_ctx_timer_start", self.h)

    def timer_stop(self) -> float:
        ms = ctypes.c_float()
        call("afem_ctx_timer_stop", self.h, ctypes.byref(ms))
        return ms.value

    def event_record(self, slot: int):
        call("afem_ctx_event_record", self.h, slot)

    def event_elapsed(self, a: int, b: int) -> float:
        ms = ctypes.c_float()
        call("afem_ctx_event_elapsed", self.h, a, b, ctypes.byref(ms))
        return ms.value

    def to_host(self, dptr: int, count: int, dtype) -> np.ndarray:
        out = np.empty(count, dtype=dtype)
        if count:
            call("afem_memcpy", self.h, _ptr(out), ctypes.c_void_p(dptr), out.nbytes, C.AFEM_MEM_HOST,
                 C.AFEM_MEM_DEVICE)
        return out

    def to_device(self, dptr: int, arr: np.ndarray):
        arr = np.ascontiguousarray(arr)
        if arr.nbytes:
            call("afem_memcpy", self.h, ctypes.c_void_p(dptr), _ptr(arr), arr.nbytes, C.AFEM_MEM_DEVICE,
                 C.AFEM_MEM_HOST)

    def malloc(self, nbytes: int) -> int:
        p = ctypes.c_void_p()
        call("afem_malloc", self.h, nbytes, ctypes.byref(p))
        return p.value

    def free(self, dptr: int):
        call("afem_free", self.h, ctypes.c_void_p(dptr))

    def close(self):
        if self.h:
            call("afem_ctx_destroy", self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def partition_rcb(dim: int, coords: np.ndarray, n_parts: int) -> np.ndarray:
    """Node partition by recursive coordinate bisection (afem_partition_rcb,
    host C++): the partitioner Arcane runs before the FEM module."""
    coords = np.ascontiguousarray(coords, dtype=np.float64).reshape(-1, 3)
    part = np.empty(coords.shape[0], dtype=np.int32)
    call("afem_partition_rcb", dim, coords.shape[0], _ptr(coords), n_parts, _ptr(part))
    return part


def subdomain_plan(cells: np.ndarray, node_part: np.ndarray, nranks: int, rank: int) -> dict:
    """Host-side subdomain plan (afem_subdomain_plan): local_to_global (owned
    then ghost nodes), cells (global ids of the local cells), neighbors and the
    send / recv lists (local node ids, split per neighbour)."""
    cells = np.ascontiguousarray(cells, dtype=np.int32)
    part = np.ascontiguousarray(node_part, dtype=np.int32)
    info = C.SubdomainInfo()
    args = (cells.shape[1], part.shape[0], cells.shape[0], _ptr(cells), _ptr(part), nranks, rank, ctypes.byref(info))
    call("afem_subdomain_plan", *args, None, None, None, None, None, None, None)
    l2g = np.empty(info.n_nodes, dtype=np.int64)
    lc = np.empty(info.n_cells, dtype=np.int64)
    nbr = np.empty(info.n_neighbors, dtype=np.int32)
    sc = np.empty(info.n_neighbors, dtype=np.int64)
    rc = np.empty(info.n_neighbors, dtype=np.int64)
    si = np.empty(info.n_send, dtype=np.int32)
    ri = np.empty(info.n_recv, dtype=np.int32)
    call("afem_subdomain_plan", *args, _ptr(l2g), _ptr(lc), _ptr(nbr), _ptr(sc), _ptr(si), _ptr(rc), _ptr(ri))
    so = np.concatenate([[0], np.cumsum(sc)]).astype(np.int64)
    ro = np.concatenate([[0], np.cumsum(rc)]).astype(np.int64)
    return dict(n_own=int(info.n_own_nodes), local_to_global=l2g, cells=lc, neighbors=nbr,
                send={int(nbr[i]): si[so[i]:so[i + 1]] for i in range(len(nbr))},
                recv={int(nbr[i]): ri[ro[i]:ro[i + 1]] for i in range(len(nbr))})


class Mesh:
    """Device-resident P1 mesh: owned nodes [0, n_own) first, then ghosts."""

    def __init__(self, ctx: Context, handle):
        self.ctx = ctx
        self.h = handle
        info = C.MeshInfo()
        call("afem_mesh_get_info", self.h, ctypes.byref(info))
        self.dim = info.dim
        self.nb_node_per_cell = info.nb_node_per_cell
        self.n_nodes = info.n_nodes
        self.n_own_nodes = info.n_own_nodes
        self.n_cells = info.n_cells

    @classmethod
    def from_arrays(cls, ctx: Context, dim: int, cells: np.ndarray, coords: np.ndarray, n_own: int | None = None):
        cells = np.ascontiguousarray(cells, dtype=np.int32)
        coords = np.ascontiguousarray(coords, dtype=np.float64).reshape(-1, 3)
        n_nodes = coords.shape[0]
        h = ctypes.c_void_p()
        call("afem_mesh_create", ctx.h, dim, cells.shape[1], n_nodes, n_nodes if n_own is None else n_own,
             cells.shape[0], _ptr(cells), _ptr(coords), C.AFEM_MEM_HOST, ctypes.byref(h))
        return cls(ctx, h)

    @classmethod
    def structured(cls, ctx: Context, dim: int, n: int, nz: int | None = None, jitter: float = 0.2,
                   seed: int = 20250220, nranks: int = 1, rank: int = 0):
        h = ctypes.c_void_p()
        call("afem_mesh_create_structured", ctx.h, dim, n, 0 if nz is None else nz, jitter, seed, nranks, rank,
             ctypes.byref(h))
        return cls(ctx, h)

    @classmethod
    def subdomain(cls, ctx: Context, dim: int, cells: np.ndarray, coords: np.ndarray, node_part: np.ndarray,
                  nranks: int, rank: int):
        """The ghosted subdomain of `rank` of a global mesh under a node
        partition (afem_mesh_create_subdomain): owned nodes first, then one
        layer of ghosts; carries its halo plan (DoFLinearSystem.set_halo_mesh)
        and its local-to-global node ids (download())."""
        cells = np.ascontiguousarray(cells, dtype=np.int32)
        coords = np.ascontiguousarray(coords, dtype=np.float64).reshape(-1, 3)
        part = np.ascontiguousarray(node_part, dtype=np.int32)
        h = ctypes.c_void_p()
        call("afem_mesh_create_subdomain", ctx.h, dim, cells.shape[1], coords.shape[0], cells.shape[0], _ptr(cells),
             _ptr(coords), _ptr(part), nranks, rank, ctypes.byref(h))
        return cls(ctx, h)

    def download(self):
        cells = np.empty((self.n_cells, self.nb_node_per_cell), dtype=np.int32)
        coords = np.empty((self.n_nodes, 3), dtype=np.float64)
        l2g = np.empty(self.n_nodes, dtype=np.int64)
        call("afem_mesh_download", self.h, _ptr(cells), _ptr(coords), _ptr(l2g))
        return cells, coords, l2g

    def bottom_nodes(self) -> np.ndarray:
        cnt = ctypes.c_int64()
        call("afem_mesh_structured_bottom_nodes", self.h, None, ctypes.byref(cnt))
        ids = np.empty(cnt.value, dtype=np.int32)
        if cnt.value:
            call("afem_mesh_structured_bottom_nodes", self.h, _ptr(ids), ctypes.byref(cnt))
        return ids

    def close(self):
        if self.h:
            call("afem_mesh_destroy", self.h)
            self.h = None


class BSRFormat:
    """BSRFormat<NB_DOF> (femutils/BSRFormat.h:353-1140)."""

    def __init__(self, mesh: Mesh, nb_dof: int = 1):
        self.mesh = mesh
        self.nb_dof = nb_dof
        self.h = None

    # BSRFormat::initialize(mesh, does_linear_system_use_csr, use_atomic_free)
    def initialize(self, use_csr_in_linear_system: bool = True):
        h = ctypes.c_void_p()
        call("afem_bsr_create", self.mesh.h, self.nb_dof, 1 if use_csr_in_linear_system else 0, ctypes.byref(h))
        self.h = h
        return self

    def computeSparsity(self):
        call("afem_bsr_compute_sparsity", self.h)

    def assemblePoissonP1(self, coef: float = 1.0, f: float | None = None, rhs_dptr: int | None = None,
                          rhs_mode: str = "add"):
        """assembleBilinear(_computeElementMatrix{Tria3,Tetra4}Gpu) fused with
        applyConstantSourceToRhs(f) into rhs_dptr when given.  rhs_mode "add"
        accumulates (the reference's atomic adds); "set" overwrites (the
        module's rhs.fill(0) + source in one pass)."""
        call("afem_bsr_assemble_poisson_p1_ex", self.h, coef, 0.0 if f is None else f,
             ctypes.c_void_p(rhs_dptr) if rhs_dptr else None, _rhs_mode(rhs_mode))

    def assembleElasticityP1(self, lam: float, mu2: float):
        call("afem_bsr_assemble_elasticity_p1", self.h, lam, mu2)

    def assembleElasticityP1Ex(self, lam: float, mu2: float, mass_coef: float = 0.0, body_force=None,
                               rhs_dptr: int | None = None, rhs_mode: str = "add"):
        """Block-3 tetrahedra: lambda/mu2 stiffness + mass_coef * consistent mass
        (Newmark LHS c0 M + K) and, with body_force (3 floats), the vectorial
        constant source into rhs_dptr (3 per owned node; rhs_mode as above)."""
        f = None
        if body_force is not None:
            f = (ctypes.c_double * 3)(*[float(x) for x in body_force])
        call("afem_bsr_assemble_elasticity_p1_ex", self.h, lam, mu2, mass_coef, f,
             ctypes.c_void_p(rhs_dptr) if rhs_dptr else None, _rhs_mode(rhs_mode))

    def resetMatrixValues(self):
        call("afem_bsr_reset_values", self.h)

    def setValue(self, row: int, col: int, v: float):
        call("afem_bsr_set_value", self.h, row, col, v)

    def getValue(self, row: int, col: int) -> float:
        v = ctypes.c_double()
        call("afem_bsr_get_value", self.h, row, col, ctypes.byref(v))
        return v.value

    def toLinearSystem(self, ls: "DoFLinearSystem"):
        call("afem_bsr_to_linear_system", self.h, ls.impl)

    def view(self) -> C.CsrView:
        v = C.CsrView()
        call("afem_bsr_view", self.h, ctypes.byref(v))
        return v

    def stats(self) -> dict:
        s = C.BsrStats()
        call("afem_bsr_get_stats", self.h, ctypes.byref(s))
        return {k: getattr(s, k) for k, _ in s._fields_}

    def functor_plan(self) -> dict:
        """The cell-unit plan of the generic element-functor kernel
        (afem_bsr_functor_plan; built at the first call)."""
        p = C.FunctorPlan()
        call("afem_bsr_functor_plan", self.h, ctypes.byref(p))
        return {k: getattr(p, k) for k, _ in p._fields_ if not k in
                ("units", "stage_ptr", "layer_rows", "entries", "entries2", "rows", "values", "stream",
                 "patterns", "reserved0")}

    def download(self):
        """Block arrays: rows[n+1] int64, columns[nnz] int32, values[nnz*k*k]."""
        v = self.view()
        rows = np.empty(v.n_block_rows + 1, dtype=np.int64)
        cols = np.empty(v.nnz_blocks, dtype=np.int32)
        vals = np.empty(v.nnz_blocks * v.block_size ** 2, dtype=np.float64)
        call("afem_bsr_download", self.h, _ptr(rows), _ptr(cols), _ptr(vals))
        return rows, cols, vals

    def export_csr32(self):
        """Scalar CSR in the reference CSRFormatView layout (BSRMatrix::toCsr)."""
        n = ctypes.c_int64()
        nnz = ctypes.c_int64()
        call("afem_bsr_get_sizes", self.h, ctypes.byref(n), ctypes.byref(nnz))
        rows = np.empty(n.value, dtype=np.int32)
        rnc = np.empty(n.value, dtype=np.int32)
        cols = np.empty(nnz.value, dtype=np.int32)
        vals = np.empty(nnz.value, dtype=np.float64)
        call("afem_bsr_export_csr32", self.h, _ptr(rows), _ptr(rnc), _ptr(cols), _ptr(vals))
        return rows, rnc, cols, vals

    def close(self):
        if self.h:
            call("afem_bsr_destroy", self.h)
            self.h = None


class DoFLinearSystem:
    """Facade of femutils/DoFLinearSystem.h:126-286 over the GPU impl."""

    def __init__(self):
        self.impl = None
        self.ctx = None
        self.factory = None
        self.n_rows = 0
        self.n_cols = 0

    def setLinearSystemFactory(self, factory: "HipDoFLinearSystemFactory"):
        self.factory = factory

    def initialize(self, ctx: Context, n_rows: int, n_cols_local: int | None = None, solver_name: str = "Solver"):
        factory = self.factory or HipDoFLinearSystemFactory()
        self.impl = factory.createInstance(ctx, n_rows, n_cols_local, solver_name)
        self.ctx = ctx
        self.n_rows = n_rows
        self.n_cols = n_rows if n_cols_local is None else n_cols_local
        return self

    def isInitialized(self) -> bool:
        return self.impl is not None

    def _check_init(self):
        if self.impl is None:
            raise AfemError(4, "DoFLinearSystem", "Linear system is not initialized (call initialize())")

    def matrixAddValue(self, row, col, v):
        self._check_init()
        call("afem_ls_matrix_add_value", self.impl, row, col, v)

    def matrixSetValue(self, row, col, v):
        self._check_init()
        call("afem_ls_matrix_set_value", self.impl, row, col, v)

    def eliminateRow(self, row, v):
        self._check_init()
        call("afem_ls_eliminate_row", self.impl, row, v)

    def eliminateRowColumn(self, row, v):
        self._check_init()
        call("afem_ls_eliminate_row_column", self.impl, row, v)

    def setCSRValues(self, rows, rows_nb_column, columns, values):
        """Host arrays in the CSRFormatView layout (rows without sentinel)."""
        self._check_init()
        rows = np.ascontiguousarray(rows, dtype=np.int32)
        columns = np.ascontiguousarray(columns, dtype=np.int32)
        values = np.ascontiguousarray(values, dtype=np.float64)
        rnc = None if rows_nb_column is None else np.ascontiguousarray(rows_nb_column, dtype=np.int32)
        call("afem_ls_set_csr_values", self.impl, _ptr(rows), None if rnc is None else _ptr(rnc), _ptr(columns),
             _ptr(values), rows.shape[0], columns.shape[0], C.AFEM_MEM_HOST)
        # the view stays the matrix until solve (libafem re-reads the values
        # then): keep the arrays alive; a float64 contiguous `values` is the
        # caller's own array, so its later edits are seen
        self._host_view = (rows, rnc, columns, values)

    def hasSetCSRValues(self) -> bool:
        self._check_init()
        h = ctypes.c_int()
        call("afem_ls_has_set_csr_values", self.impl, ctypes.byref(h))
        return bool(h.value)

    def getCSRValues(self) -> C.CsrView:
        self._check_init()
        v = C.CsrView()
        call("afem_ls_get_csr_values", self.impl, ctypes.byref(v))
        return v

    def _dptr(self, name):
        p = ctypes.c_void_p()
        call(name, self.impl, ctypes.byref(p))
        return p.value

    # device addresses of the impl-owned variables
    def rhsVariable(self) -> int:
        return self._dptr("afem_ls_rhs")

    def solutionVariable(self) -> int:
        return self._dptr("afem_ls_solution")

    def getForcedInfo(self) -> int:
        return self._dptr("afem_ls_forced_info")

    def getForcedValue(self) -> int:
        return self._dptr("afem_ls_forced_value")

    def getEliminationInfo(self) -> int:
        return self._dptr("afem_ls_elimination_info")

    def getEliminationValue(self) -> int:
        return self._dptr("afem_ls_elimination_value")

    def rhs_host(self):
        return self.ctx.to_host(self.rhsVariable(), self.n_rows, np.float64)

    def set_rhs_host(self, b):
        self.ctx.to_device(self.rhsVariable(), np.asarray(b, dtype=np.float64))

    def solution_host(self, with_ghosts=False):
        return self.ctx.to_host(self.solutionVariable(), self.n_cols if with_ghosts else self.n_rows, np.float64)

    def applyDirichletViaPenalty(self, dofs, value: float, penalty: float = 1.0e30):
        """Gpu::BoundaryConditionsHelpers::applyDirichletToNodeGroupViaPenalty."""
        self._check_init()
        dofs = np.ascontiguousarray(dofs, dtype=np.int32)
        call("afem_ls_dirichlet_penalty", self.impl, _ptr(dofs), dofs.shape[0], value, penalty, C.AFEM_MEM_HOST)

    def applyDirichletViaPenaltyDevice(self, dofs_dptr: int, n: int, value: float, penalty: float = 1.0e30):
        """Same, with the DoF list already resident in device memory (no copy)."""
        self._check_init()
        call("afem_ls_dirichlet_penalty", self.impl, ctypes.c_void_p(dofs_dptr), n, value, penalty,
             C.AFEM_MEM_DEVICE)

    def applyDirichletViaRowElimination(self, dofs, value: float):
        self._check_init()
        dofs = np.ascontiguousarray(dofs, dtype=np.int32)
        call("afem_ls_dirichlet_row_elimination", self.impl, _ptr(dofs), dofs.shape[0], value, C.AFEM_MEM_HOST)

    def applyBoundaryConditions(self):
        call("afem_ls_apply_boundary_conditions", self.impl)

    SOLVERS = {"auto": C.AFEM_SOLVER_AUTO, "pcg": C.AFEM_SOLVER_PCG, "direct": C.AFEM_SOLVER_DIRECT}

    def setSolverOptions(self, rtol=None, atol=None, max_iter=None, check_every=None, fixed_iterations=None,
                         method=None, initial_guess=None, preconditioner=None, profile_comm=None):
        """initial_guess: "zero" (default) or "current" (start the PCG from the
        solution vector's values); preconditioner: "jacobi" (default),
        "block3" (3x3 node-block Jacobi, NB_DOF = 3 systems), "multigrid"
        (geometric multigrid V-cycle on structured boxes, one rank or z-slabs; rebuilt
        every solve), "multigrid-reuse" (built once, reused while the
        matrix structure is unchanged), "amg" / "amg-reuse" (algebraic
        multigrid from the CSR: any mesh, one rank) or "multigrid+amg" (the
        geometric hierarchy where it exists, else the algebraic one)."""
        o = C.SolverOpts()
        call("afem_ls_get_solver_options", self.impl, ctypes.byref(o))
        if method is not None:
            o.method = self.SOLVERS[method]
        if rtol is not None:
            o.rtol = rtol
        if atol is not None:
            o.atol = atol
        if max_iter is not None:
            o.max_iter = max_iter
        if check_every is not None:
            o.check_every = check_every
        if fixed_iterations is not None:
            o.fixed_iterations = fixed_iterations
        if profile_comm is not None:
            o.profile_comm = 1 if profile_comm else 0
        if initial_guess is not None:
            o.initial_guess = {"zero": 0, "current": 1}[initial_guess]
        if preconditioner is not None:
            o.precond_block, o.multigrid, o.amg = {
                "jacobi": (0, 0, 0), "block3": (3, 0, 0), "multigrid": (0, 1, 0), "multigrid-reuse": (0, 2, 0),
                "amg": (0, 0, 1), "amg-reuse": (0, 0, 2), "multigrid+amg": (0, 1, 1)}[preconditioner]
        call("afem_ls_set_solver_options", self.impl, ctypes.byref(o))

    def solve(self) -> dict:
        self._check_init()
        st = C.SolveStats()
        call("afem_ls_solve", self.impl, ctypes.byref(st))
        return dict(iterations=st.iterations, converged=bool(st.converged), rel_residual=st.rel_residual,
                    residual_norm=st.residual_norm, solve_ms=st.solve_ms, spmv_kernel=st.spmv_kernel,
                    halo_wait_ms=st.halo_wait_ms, allreduce_ms=st.allreduce_ms, halo_bytes=st.halo_bytes,
                    n_halo=st.n_halo, n_allreduce=st.n_allreduce, amg_levels=st.amg_levels,
                    amg_coarse_rows=st.amg_coarse_rows, amg_complexity=st.amg_complexity,
                    amg_setup_ms=st.amg_setup_ms, precond_ms=st.precond_ms)

    def spmv(self, x_dptr: int, y_dptr: int):
        call("afem_ls_spmv", self.impl, ctypes.c_void_p(x_dptr), ctypes.c_void_p(y_dptr))

    def clearValues(self):
        self._check_init()
        call("afem_ls_clear_values", self.impl)
        self._host_view = None

    def set_halo(self, comm, neighbors, send_ids, recv_ids):
        """afem_ls_set_halo from the caller's own synchronisation lists (what
        an Arcane shim builds from the DoF family's IVariableSynchronizer,
        femutils/FemDoFsOnNodes.cc:125-126): for each neighbour rank (in order)
        the owned DoFs to send and the ghost DoFs (ids >= n_rows) to receive."""
        nbr = np.ascontiguousarray(neighbors, dtype=np.int32)
        sl = [np.ascontiguousarray(a, dtype=np.int32) for a in send_ids]
        rl = [np.ascontiguousarray(a, dtype=np.int32) for a in recv_ids]
        if len(sl) != nbr.size or len(rl) != nbr.size:
            raise ValueError("one send and one receive list per neighbour")
        sc = np.array([a.size for a in sl], dtype=np.int64)
        rc = np.array([a.size for a in rl], dtype=np.int64)
        si = np.concatenate(sl + [np.zeros(1, np.int32)])  # never empty: a valid pointer
        ri = np.concatenate(rl + [np.zeros(1, np.int32)])
        call("afem_ls_set_halo", self.impl, comm.h, nbr.size, _ptr(nbr) if nbr.size else None,
             _ptr(sc) if nbr.size else None, _ptr(si), _ptr(rc) if nbr.size else None, _ptr(ri))

    def set_halo_structured(self, comm, mesh: Mesh):
        call("afem_ls_set_halo_structured", self.impl, comm.h, mesh.h)

    def set_halo_mesh(self, comm, mesh: Mesh):
        """Halo plan of a structured slab or a partitioned subdomain (NB_DOF-aware)."""
        call("afem_ls_set_halo_mesh", self.impl, comm.h, mesh.h)

    def synchronize(self, x_dptr: int):
        call("afem_ls_synchronize", self.impl, ctypes.c_void_p(x_dptr))

    def reset(self):
        if self.impl:
            call("afem_ls_destroy", self.impl)
            self.impl = None

    def __del__(self):
        try:
            self.reset()
        except Exception:
            pass


class HipDoFLinearSystemFactory:
    """IDoFLinearSystemFactory::createInstance -> a GPU DoFLinearSystemImpl."""

    service_name = "HipLinearSystem"

    def createInstance(self, ctx: Context, n_rows: int, n_cols_local: int | None = None, solver_name: str = "Solver"):
        h = ctypes.c_void_p()
        call("afem_ls_create", ctx.h, n_rows, n_rows if n_cols_local is None else n_cols_local, ctypes.byref(h))
        return h


class Communicator:
    """RCCL communicator of the data path; bootstrapped through any object
    with a ``broadcast_bytes(buf, root)`` (the torch.distributed helper in
    parallel.py)."""

    def __init__(self, ctx: Context, nranks: int, rank: int, unique_id: bytes):
        idb = (ctypes.c_uint8 * C.UNIQUE_ID_BYTES).from_buffer_copy(unique_id.ljust(C.UNIQUE_ID_BYTES, b"\0"))
        h = ctypes.c_void_p()
        call("afem_comm_create", ctx.h, idb, nranks, rank, ctypes.byref(h))
        self.h = h
        self.nranks = nranks
        self.rank = rank

    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_uint8 * C.UNIQUE_ID_BYTES)()
        call("afem_comm_unique_id", buf)
        return bytes(buf)

    def close(self):
        if self.h:
            call("afem_comm_destroy", self.h)
            self.h = None


def structured_halo_plan(dim, n, nz, nranks, rank):
    """Host-only: (neighbour ranks, send_counts, recv_counts, send_ids, recv_ids)."""
    nn = ctypes.c_int()
    call("afem_structured_halo_plan", dim, n, nz or 0, nranks, rank, ctypes.byref(nn), None, None, None, None, None)
    k = nn.value
    nbr = np.zeros(max(k, 1), dtype=np.int32)
    sc = np.zeros(max(k, 1), dtype=np.int64)
    rc = np.zeros(max(k, 1), dtype=np.int64)
    call("afem_structured_halo_plan", dim, n, nz or 0, nranks, rank, ctypes.byref(nn), _ptr(nbr), _ptr(sc), _ptr(rc),
         None, None)
    si = np.zeros(max(int(sc[:k].sum()), 1), dtype=np.int32)
    ri = np.zeros(max(int(rc[:k].sum()), 1), dtype=np.int32)
    call("afem_structured_halo_plan", dim, n, nz or 0, nranks, rank, ctypes.byref(nn), _ptr(nbr), _ptr(sc), _ptr(rc),
         _ptr(si), _ptr(ri))
    return nbr[:k], sc[:k], rc[:k], si[:int(sc[:k].sum())], ri[:int(rc[:k].sum())]
