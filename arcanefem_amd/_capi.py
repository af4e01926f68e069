"""ctypes binding of include/arcanefem_amd.h (libafem.so, built in-tree).

The product path has no fallback: if the HIP library is missing or fails to
load, every call raises.  Python is the host driver only; all compute runs in
libafem.so on the GPU.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("AFEM_LIB") or os.path.join(_HERE, "libafem.so")  # AFEM_LIB: diagnostic builds

AFEM_OK = 0
AFEM_MEM_HOST = 0
AFEM_MEM_DEVICE = 1
AFEM_RHS_ADD = 0
AFEM_RHS_SET = 1
AFEM_SOLVER_AUTO = 0
AFEM_SOLVER_PCG = 1
AFEM_SOLVER_DIRECT = 2
AFEM_NEUMANN_VALUE = 0
AFEM_NEUMANN_NORMAL = 1
AFEM_NEUMANN_TRACTION = 2
UNIQUE_ID_BYTES = 128
ERRORS = {1: "ArgumentException", 2: "HipError", 3: "NotImplementedException", 4: "StateError",
          5: "NotFound", 6: "CommError", 7: "LimitExceeded"}


class AfemError(RuntimeError):
    def __init__(self, code, func, msg):
        self.code = code
        super().__init__(f"{func}: [{ERRORS.get(code, code)}] {msg}")


class MeshInfo(ctypes.Structure):
    _fields_ = [("dim", ctypes.c_int32), ("nb_node_per_cell", ctypes.c_int32), ("n_nodes", ctypes.c_int64),
                ("n_own_nodes", ctypes.c_int64), ("n_cells", ctypes.c_int64)]


class SubdomainInfo(ctypes.Structure):
    _fields_ = [("n_own_nodes", ctypes.c_int64), ("n_nodes", ctypes.c_int64), ("n_cells", ctypes.c_int64),
                ("n_neighbors", ctypes.c_int), ("n_send", ctypes.c_int64), ("n_recv", ctypes.c_int64)]


class CsrView(ctypes.Structure):
    _fields_ = [("n_block_rows", ctypes.c_int64), ("n_block_cols", ctypes.c_int64), ("nnz_blocks", ctypes.c_int64),
                ("block_size", ctypes.c_int32), ("ordered_per_block", ctypes.c_int32), ("rows", ctypes.c_void_p),
                ("columns", ctypes.c_void_p), ("values", ctypes.c_void_p)]


class AssemblyView(ctypes.Structure):
    """afem_assembly_view (device pointers of a structure for generic element-functor assembly)."""
    _fields_ = [("n_rows", ctypes.c_int64), ("n_nodes", ctypes.c_int64), ("n_cells", ctypes.c_int64),
                ("nb_node_per_cell", ctypes.c_int32), ("block_size", ctypes.c_int32),
                ("ordered_per_block", ctypes.c_int32), ("dim", ctypes.c_int32), ("cell_node", ctypes.c_void_p),
                ("coords", ctypes.c_void_p), ("rows", ctypes.c_void_p), ("columns", ctypes.c_void_p),
                ("values", ctypes.c_void_p), ("error_flag", ctypes.c_void_p), ("stream", ctypes.c_void_p)]


class FunctorPlan(ctypes.Structure):
    """afem_functor_plan (cell-unit plan of the generic element-functor kernel)."""
    _fields_ = [("n_units", ctypes.c_int64), ("n_stages", ctypes.c_int64), ("n_entries", ctypes.c_int64),
                ("rows_per_layer", ctypes.c_int32), ("width", ctypes.c_int32), ("nbuf", ctypes.c_int32),
                ("wide", ctypes.c_int32), ("block_size", ctypes.c_int32), ("nb_node_per_cell", ctypes.c_int32),
                ("ordered_per_block", ctypes.c_int32), ("lattice", ctypes.c_int32), ("units", ctypes.c_void_p),
                ("stage_ptr", ctypes.c_void_p), ("layer_rows", ctypes.c_void_p), ("entries", ctypes.c_void_p),
                ("entries2", ctypes.c_void_p), ("rows", ctypes.c_void_p), ("values", ctypes.c_void_p),
                ("stream", ctypes.c_void_p), ("patterns", ctypes.c_void_p), ("n_patterns", ctypes.c_int64),
                ("packed", ctypes.c_int32), ("reserved0", ctypes.c_int32)]


class Csr32View(ctypes.Structure):
    """afem_csr32_view (BSRFormat::toLinearSystem in the caller's DoF numbering)."""
    _fields_ = [("n_rows", ctypes.c_int64), ("nnz", ctypes.c_int64), ("rows", ctypes.c_void_p),
                ("rows_nb_column", ctypes.c_void_p), ("columns", ctypes.c_void_p), ("values", ctypes.c_void_p),
                ("identity", ctypes.c_int32)]


class BsrStats(ctypes.Structure):
    _fields_ = [("n_incidences", ctypes.c_int64), ("inc_table_entries", ctypes.c_int64),
                ("max_row_len", ctypes.c_int32), ("rows_per_block", ctypes.c_int32), ("max_seg", ctypes.c_int64),
                ("max_slice_nodes", ctypes.c_int32), ("max_slice_width", ctypes.c_int32),
                ("n_slices", ctypes.c_int64), ("brick_order", ctypes.c_int32), ("uniform_slices", ctypes.c_int32),
                ("last_kernel", ctypes.c_int32), ("stencil_slices", ctypes.c_int32),
                ("stencil_sig", ctypes.c_int32), ("shared_strip_slices", ctypes.c_int64),
                ("uniform_instance_slices", ctypes.c_int64), ("general_slices", ctypes.c_int64),
                ("cube_lattice", ctypes.c_int32), ("cube_axes", ctypes.c_int32)]


class SolverOpts(ctypes.Structure):
    _fields_ = [("method", ctypes.c_int32), ("max_iter", ctypes.c_int32), ("rtol", ctypes.c_double),
                ("atol", ctypes.c_double), ("check_every", ctypes.c_int32), ("fixed_iterations", ctypes.c_int32),
                ("initial_guess", ctypes.c_int32), ("precond_block", ctypes.c_int32), ("multigrid", ctypes.c_int32),
                ("profile_comm", ctypes.c_int32), ("amg", ctypes.c_int32)]


class SolveStats(ctypes.Structure):
    _fields_ = [("iterations", ctypes.c_int32), ("converged", ctypes.c_int32), ("rel_residual", ctypes.c_double),
                ("residual_norm", ctypes.c_double), ("solve_ms", ctypes.c_double), ("spmv_kernel", ctypes.c_int32),
                ("halo_wait_ms", ctypes.c_double), ("allreduce_ms", ctypes.c_double), ("halo_bytes", ctypes.c_int64),
                ("n_halo", ctypes.c_int32), ("n_allreduce", ctypes.c_int32), ("amg_levels", ctypes.c_int32),
                ("amg_coarse_rows", ctypes.c_int64), ("amg_complexity", ctypes.c_double),
                ("amg_setup_ms", ctypes.c_double), ("precond_ms", ctypes.c_double)]


class StepTiming(ctypes.Structure):
    _fields_ = [("assemble_ms", ctypes.c_double), ("rhs_ms", ctypes.c_double), ("bc_ms", ctypes.c_double),
                ("solve_ms", ctypes.c_double), ("precond_ms", ctypes.c_double), ("update_ms", ctypes.c_double),
                ("total_ms", ctypes.c_double), ("iterations", ctypes.c_int32), ("reserved0", ctypes.c_int32),
                ("nnz_blocks", ctypes.c_int64), ("n_incidences", ctypes.c_int64), ("n_nodes", ctypes.c_int64),
                ("n_own_nodes", ctypes.c_int64)]


ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int64)
EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int32),
                               ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64),
                               ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64))


class HostTransport(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("allreduce_sum", ALLREDUCE_FN), ("exchange", EXCHANGE_FN)]


class NewmarkParams(ctypes.Structure):
    _fields_ = [("E", ctypes.c_double), ("nu", ctypes.c_double), ("rho", ctypes.c_double), ("dt", ctypes.c_double),
                ("body_force", ctypes.c_double * 3), ("penalty", ctypes.c_double), ("gamma", ctypes.c_double),
                ("beta", ctypes.c_double), ("etam", ctypes.c_double), ("etak", ctypes.c_double),
                ("alpm", ctypes.c_double), ("alpf", ctypes.c_double), ("scheme", ctypes.c_int32),
                ("reserved0", ctypes.c_int32)]


P = ctypes.c_void_p
PP = ctypes.POINTER(ctypes.c_void_p)
I32 = ctypes.c_int32
I64 = ctypes.c_int64
U64 = ctypes.c_uint64
D = ctypes.c_double
INT = ctypes.c_int

# name -> argtypes (all return int status, except afem_last_error / afem_version)
SIGNATURES = {
    "afem_device_count": [ctypes.POINTER(INT)],
    "afem_set_variant": [ctypes.c_char_p, ctypes.c_char_p],
    "afem_ctx_create": [INT, P, PP],
    "afem_ctx_destroy": [P],
    "afem_ctx_synchronize": [P],
    "afem_ctx_stream": [P, PP],
    "afem_ctx_timer_start": [P],
    "afem_ctx_timer_stop": [P, ctypes.POINTER(ctypes.c_float)],
    "afem_ctx_event_record": [P, INT],
    "afem_ctx_event_elapsed": [P, INT, INT, ctypes.POINTER(ctypes.c_float)],
    "afem_malloc": [P, ctypes.c_size_t, PP],
    "afem_free": [P, P],
    "afem_memcpy": [P, P, P, ctypes.c_size_t, INT, INT],
    "afem_mesh_create": [P, INT, INT, I64, I64, I64, P, P, INT, PP],
    "afem_mesh_create_structured": [P, INT, INT, INT, D, U64, INT, INT, PP],
    "afem_mesh_get_info": [P, ctypes.POINTER(MeshInfo)],
    "afem_partition_rcb": [INT, I64, P, INT, P],
    "afem_subdomain_plan": [INT, I64, I64, P, P, INT, INT, ctypes.POINTER(SubdomainInfo), P, P, P, P, P, P, P],
    "afem_mesh_create_subdomain": [P, INT, INT, I64, I64, P, P, P, INT, INT, PP],
    "afem_mesh_download": [P, P, P, P],
    "afem_mesh_structured_bottom_nodes": [P, P, ctypes.POINTER(I64)],
    "afem_mesh_destroy": [P],
    "afem_bsr_create": [P, INT, INT, PP],
    "afem_bsr_compute_sparsity": [P],
    "afem_bsr_assemble_poisson_p1": [P, D, D, P],
    "afem_bsr_assemble_poisson_p1_ex": [P, D, D, P, INT],
    "afem_bsr_assemble_elasticity_p1": [P, D, D],
    "afem_bsr_assemble_elasticity_p1_ex": [P, D, D, D, P, P, INT],
    "afem_apply_neumann": [P, INT, INT, P, I64, P, P, INT, P],
    "afem_vec_lincomb": [P, I64, D, P, D, P, D, P, P],
    "afem_newmark_update": [P, I64, D, D, D, P, P, P, P],
    "afem_bsr_reset_values": [P],
    "afem_bsr_set_value": [P, I32, I32, D],
    "afem_bsr_get_value": [P, I32, I32, ctypes.POINTER(D)],
    "afem_bsr_view": [P, ctypes.POINTER(CsrView)],
    "afem_bsr_get_stats": [P, ctypes.POINTER(BsrStats)],
    "afem_bsr_assembly_view": [P, ctypes.POINTER(AssemblyView)],
    "afem_bsr_functor_plan": [P, ctypes.POINTER(FunctorPlan)],
    "afem_bsr_to_csr32_mapped": [P, P, I64, ctypes.POINTER(Csr32View)],
    "afem_bsr_get_sizes": [P, ctypes.POINTER(I64), ctypes.POINTER(I64)],
    "afem_bsr_export_csr32": [P, P, P, P, P],
    "afem_bsr_download": [P, P, P, P],
    "afem_bsr_to_linear_system": [P, P],
    "afem_bsr_destroy": [P],
    "afem_ls_create": [P, I64, I64, PP],
    "afem_ls_set_solver_options": [P, ctypes.POINTER(SolverOpts)],
    "afem_ls_get_solver_options": [P, ctypes.POINTER(SolverOpts)],
    "afem_ls_matrix_add_value": [P, I32, I32, D],
    "afem_ls_matrix_set_value": [P, I32, I32, D],
    "afem_ls_eliminate_row": [P, I32, D],
    "afem_ls_eliminate_row_column": [P, I32, D],
    "afem_ls_set_csr_values": [P, P, P, P, P, I32, I32, INT],
    "afem_ls_set_csr_values_mapped": [P, P, P, P, P, I32, I32, P, I64],
    "afem_ls_has_set_csr_values": [P, ctypes.POINTER(INT)],
    "afem_ls_get_csr_values": [P, ctypes.POINTER(CsrView)],
    "afem_ls_rhs": [P, PP],
    "afem_ls_solution": [P, PP],
    "afem_ls_forced_info": [P, PP],
    "afem_ls_forced_value": [P, PP],
    "afem_ls_elimination_info": [P, PP],
    "afem_ls_elimination_value": [P, PP],
    "afem_ls_dirichlet_penalty": [P, P, I64, D, D, INT],
    "afem_ls_dirichlet_row_elimination": [P, P, I64, D, INT],
    "afem_ls_apply_boundary_conditions": [P],
    "afem_ls_clear_values": [P],
    "afem_ls_solve": [P, ctypes.POINTER(SolveStats)],
    "afem_ls_spmv": [P, P, P],
    "afem_ls_destroy": [P],
    "afem_comm_unique_id": [P],
    "afem_comm_create": [P, P, INT, INT, PP],
    "afem_comm_create_host": [P, INT, INT, ctypes.POINTER(HostTransport), PP],
    "afem_elastodynamics_create": [P, P, ctypes.POINTER(NewmarkParams), P, I64, INT, PP],
    "afem_elastodynamics_set_solver_options": [P, ctypes.POINTER(SolverOpts)],
    "afem_elastodynamics_step": [P, ctypes.POINTER(SolveStats)],
    "afem_elastodynamics_set_dirichlet": [P, P, P, I64, INT],
    "afem_elastodynamics_set_time_step": [P, D],
    "afem_elastodynamics_state": [P, PP, PP, PP],
    "afem_elastodynamics_operators": [P, ctypes.POINTER(CsrView), PP, PP, PP, P],
    "afem_elastodynamics_profile": [P, INT],
    "afem_elastodynamics_step_timing": [P, ctypes.POINTER(StepTiming)],
    "afem_elastodynamics_destroy": [P],
    "afem_comm_host_async": [P, INT],
    "afem_comm_destroy": [P],
    "afem_comm_allreduce_sum": [P, P, I64],
    "afem_ls_set_halo": [P, P, INT, P, P, P, P, P],
    "afem_ls_set_halo_structured": [P, P, P],
    "afem_ls_set_halo_mesh": [P, P, P],
    "afem_structured_halo_plan": [INT, INT, INT, INT, INT, ctypes.POINTER(INT), P, P, P, P, P],
    "afem_ls_synchronize": [P, P],
}

_lib = None


def load():
    """Load libafem.so (raises OSError if it was not built: no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                          "or `make -C arcanefem_amd/csrc`")
        L = ctypes.CDLL(LIB_PATH)
        L.afem_last_error.restype = ctypes.c_char_p
        L.afem_last_error.argtypes = []
        L.afem_version.restype = ctypes.c_int
        L.afem_version.argtypes = []
        for name, args in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = ctypes.c_int
            f.argtypes = args
        _lib = L
    return _lib


def call(name, *args):
    L = load()
    rc = getattr(L, name)(*args)
    if rc != AFEM_OK:
        raise AfemError(rc, name, L.afem_last_error().decode(errors="replace"))
    return rc


def exported_symbols():
    return ["afem_last_error", "afem_version"] + list(SIGNATURES)
