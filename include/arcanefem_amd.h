/*
 * arcanefem_amd.h — C ABI of the MI355X-native FEM assembly + CG path.
 *
 * This is the drop-in boundary for the reference's linear-system plugin
 * surface (toutane/arcanefem @ 2025-02-20, paths relative to its root):
 *
 *   DoFLinearSystemImpl        femutils/DoFLinearSystem.h:84-110   -> afem_ls_*
 *   IDoFLinearSystemFactory    femutils/IDoFLinearSystemFactory.h:34-44
 *                                                                  -> afem_ls_create
 *   CSRFormatView              femutils/DoFLinearSystem.h:42-76    -> afem_csr_view
 *   BSRFormat<NB_DOF>          femutils/BSRFormat.h:353-1140       -> afem_bsr_*
 *   FemDoFsOnNodes             femutils/FemDoFsOnNodes.cc:71-128   -> DoF lid = node_lid*k + i
 *   Gpu BC kernels             femutils/ArcaneFemFunctionsGpu.h:401-482
 *                                                                  -> afem_ls_dirichlet_* / afem_bsr_assemble_*
 *
 * Conventions
 *   - Every function returns AFEM_OK (0) or an AFEM_ERR_* code and never
 *     throws; afem_last_error() returns the thread-local message of the last
 *     failure (the reference raises ARCANE_FATAL / NotImplementedException /
 *     ArgumentException; the same conditions map to the codes below).
 *   - Handles are opaque; the caller owns them and releases them with the
 *     matching *_destroy.  Device arrays returned by *_view / *_rhs / ... are
 *     owned by the handle and stay valid until it is destroyed (or, for a CSR
 *     view, until the structure is recomputed).
 *   - Pointers passed with mem == AFEM_MEM_HOST are host memory and are copied;
 *     with AFEM_MEM_DEVICE they are device pointers on the handle's device.
 *   - All device work of a handle is enqueued on its context's HIP stream;
 *     functions that return host data synchronise that stream.
 *   - Index types: DoF / node / cell local ids are int32 (as the reference's
 *     Int32 local ids); row offsets are int64 internally so a single
 *     subdomain may exceed 2^31 non-zeros (288 GB of HBM allows ~1e9 DoF).
 *   - One host thread drives one handle (the reference is not thread-safe
 *     either, SURVEY.md §8b "Threading").
 */
#ifndef ARCANEFEM_AMD_H
#define ARCANEFEM_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AFEM_OK 0
#define AFEM_ERR_ARG 1        /* ArgumentException */
#define AFEM_ERR_HIP 2        /* HIP runtime / device failure */
#define AFEM_ERR_NOT_IMPL 3   /* NotImplementedException */
#define AFEM_ERR_STATE 4      /* call out of order (e.g. assemble before sparsity) */
#define AFEM_ERR_NOT_FOUND 5  /* (row,col) not in the sparsity (BSRMatrix::findValueIndex throws) */
#define AFEM_ERR_COMM 6       /* RCCL failure */
#define AFEM_ERR_LIMIT 7      /* an implementation limit was exceeded (message says which) */

#define AFEM_MEM_HOST 0
#define AFEM_MEM_DEVICE 1

typedef struct afem_ctx afem_ctx;   /* device + HIP stream (+ timing events) */
typedef struct afem_mesh afem_mesh; /* device-resident P1 mesh (Arcane IMesh subset) */
typedef struct afem_bsr afem_bsr;   /* BSRFormat<NB_DOF> */
typedef struct afem_ls afem_ls;     /* DoFLinearSystemImpl */
typedef struct afem_comm afem_comm; /* RCCL communicator (IParallelMng subset) */

/* ---------------------------------------------------------------- basics */
const char* afem_last_error(void);
int afem_version(void); /* major*10000 + minor*100 + patch */
int afem_device_count(int* count);
/* Kernel-variant knobs, for diagnostics and A/B measurements:
 * name "AFEM_*", value a string, NULL to return to the default.  Knobs:
 * AFEM_ASSEMBLY_STENCIL / _UNIFORM / _STRIPS / _SIDE / _WAVES_PER_CU,
 * AFEM_ELAST_WG / _STRIP / _BIG (assembly instances), AFEM_SPMV (CG SpMV),
 * AFEM_CG_GRAPH (1: replay the single-rank CG iterations as a HIP graph; off by
 * default, slower on MI355X),
 * AFEM_ORDER / AFEM_BRICKS / AFEM_BANK_PLACE / _MAX (structure build),
 * AFEM_MG_F32 / _FUSE / _KCYCLE / _OMEGA, AFEM_AMG_F32 / _FUSE / _KCYCLE /
 * _POWER_ITS / _OMEGA / _VERBOSE and the other AFEM_AMG_* setup knobs
 * (preconditioners: the fp32 cycle products and the smoother's omega change
 * the preconditioner, never the PCG's own fp64 product or its tolerance),
 * AFEM_DEBUG_SLICES / _PATTERNS (stderr dumps).  Without an explicit value a
 * knob takes the process environment's value at its first use; unset means
 * the default variant, which is what every result in DESIGN.md used.  The
 * variant that ran is reported (afem_bsr_stats.last_kernel,
 * afem_solve_stats.spmv_kernel); every variant gives the oracle's values. */
int afem_set_variant(const char* name, const char* value);

/* ---------------------------------------------------------------- context */
/* hip_stream may be NULL: the context then creates and owns a non-blocking
 * stream on `device`. */
int afem_ctx_create(int device, void* hip_stream, afem_ctx** out);
int afem_ctx_destroy(afem_ctx* ctx);
int afem_ctx_synchronize(afem_ctx* ctx);
int afem_ctx_stream(afem_ctx* ctx, void** hip_stream);
/* Event timing on the context stream: afem_ctx_timer_start(), enqueue work,
 * afem_ctx_timer_stop(&ms) (synchronises). */
int afem_ctx_timer_start(afem_ctx* ctx);
int afem_ctx_timer_stop(afem_ctx* ctx, float* ms);
/* Event pool (AFEM_EVENT_SLOTS events per context) for timing individual
 * launches inside a pipelined region without synchronising: record slots on
 * the context stream, read the elapsed time between two slots afterwards
 * (afem_ctx_event_elapsed waits for the later one). */
#define AFEM_EVENT_SLOTS 256
int afem_ctx_event_record(afem_ctx* ctx, int slot);
int afem_ctx_event_elapsed(afem_ctx* ctx, int slot_a, int slot_b, float* ms);
/* Device memory helpers for callers without their own allocator. */
int afem_malloc(afem_ctx* ctx, size_t bytes, void** dptr);
int afem_free(afem_ctx* ctx, void* dptr);
int afem_memcpy(afem_ctx* ctx, void* dst, const void* src, size_t bytes, int dst_mem, int src_mem);

/* ---------------------------------------------------------------- mesh */
typedef struct afem_mesh_info {
  int32_t dim;           /* 2 or 3 */
  int32_t nb_node_per_cell; /* 3 (TRIA3) or 4 (TETRA4) */
  int64_t n_nodes;       /* local nodes: owned first, then ghosts */
  int64_t n_own_nodes;   /* nodes [0, n_own_nodes) are owned (isOwn()) */
  int64_t n_cells;       /* local cells (own + one ghost layer) */
} afem_mesh_info;

/* Mesh from caller arrays: cell_node[n_cells*nv] (int32 local node ids, nodes
 * [0,n_own_nodes) owned) and coords[n_nodes*3] (x,y,z per node, the layout of
 * Arcane's VariableNodeReal3). */
int afem_mesh_create(afem_ctx* ctx, int dim, int nb_node_per_cell, int64_t n_nodes, int64_t n_own_nodes,
                     int64_t n_cells, const int32_t* cell_node, const double* coords, int mem, afem_mesh** out);
/* Synthetic jittered structured mesh generated on the device (DESIGN.md
 * "Synthetic inputs"): unit square split in 2 triangles per square (dim 2)
 * or box [0,1]^2 x [0,nz/n] split in 6 Kuhn tetrahedra per cube (dim 3),
 * coordinate jitter uniform in +-jitter*h/2, seeded hash.  The global mesh is
 * cut in `nranks` slabs along the last axis and this call builds the slab of
 * `rank` with one ghost node/cell layer (nranks = 1: the whole mesh). */
int afem_mesh_create_structured(afem_ctx* ctx, int dim, int n, int nz, double jitter, uint64_t seed, int nranks,
                                int rank, afem_mesh** out);
/* ---- partitioned general meshes (Gmsh): what Arcane does before the FEM
 * module sees the mesh (partitioner + one ghost layer) and what
 * femutils/FemDoFsOnNodes.cc:71-128 does after it (DoF owner = node owner,
 * computeSynchronizeInfos: the send / receive lists).  Host-side, C++. */
/* Recursive coordinate bisection of the nodes into n_parts parts (node counts
 * proportional, compact, deterministic).  coords[n_nodes*3]; node_part out. */
int afem_partition_rcb(int dim, int64_t n_nodes, const double* coords, int n_parts, int32_t* node_part);
typedef struct afem_subdomain_info {
  int64_t n_own_nodes, n_nodes, n_cells; /* local: owned nodes first, then ghosts */
  int n_neighbors;
  int64_t n_send, n_recv;
} afem_subdomain_info;
/* The subdomain of `rank` for a node partition of a global mesh (host arrays):
 * owned nodes (node_part == rank) then the ghost nodes (the other nodes of
 * every cell with an owned node), each in global order; the local cells
 * (every cell with an owned node, global order); per neighbour rank
 * (ascending) the owned nodes that are ghosts there (send) and the ghosts it
 * owns (receive), local ids in global order: rank r's send list to s is rank
 * s's receive list from r.  Output arrays may be NULL (sizes in *info). */
int afem_subdomain_plan(int nb_node_per_cell, int64_t n_nodes, int64_t n_cells, const int32_t* cell_node,
                        const int32_t* node_part, int nranks, int rank, afem_subdomain_info* info,
                        int64_t* local_to_global, int64_t* cells, int32_t* neighbor_ranks, int64_t* send_counts,
                        int32_t* send_ids, int64_t* recv_counts, int32_t* recv_ids);
/* The local mesh of that subdomain (afem_mesh_create on the local arrays); it
 * keeps its halo plan (afem_ls_set_halo_mesh) and local_to_global
 * (afem_mesh_download). */
int afem_mesh_create_subdomain(afem_ctx* ctx, int dim, int nb_node_per_cell, int64_t n_nodes, int64_t n_cells,
                               const int32_t* cell_node, const double* coords, const int32_t* node_part, int nranks,
                               int rank, afem_mesh** out);
int afem_mesh_get_info(const afem_mesh* mesh, afem_mesh_info* info);
/* Copies to host: cell_node[n_cells*nv], coords[n_nodes*3], local_to_global[n_nodes]
 * (any pointer may be NULL). local_to_global is the identity for meshes from
 * afem_mesh_create. */
int afem_mesh_download(afem_mesh* mesh, int32_t* cell_node, double* coords, int64_t* local_to_global);
/* Structured meshes: local ids of the owned nodes on the z = 0 face (y = 0 in
 * 2D), i.e. the Dirichlet group of the benchmark configs.  *count receives the
 * size; ids may be NULL to query it. */
int afem_mesh_structured_bottom_nodes(afem_mesh* mesh, int32_t* ids, int64_t* count);
int afem_mesh_destroy(afem_mesh* mesh);

/* ---------------------------------------------------------------- BSRFormat */
/* CSR / BSR arrays (device pointers).  rows[n_block_rows+1] has the n+1
 * sentinel (the reference's CSRFormatView::rows has none, its row end is
 * derived, femutils/HypreDoFLinearSystem.cc:140-141; afem_bsr_export_csr32
 * produces exactly that layout).  Columns are sorted ascending within a row. */
typedef struct afem_csr_view {
  int64_t n_block_rows;
  int64_t n_block_cols;  /* local columns (owned + ghost nodes) */
  int64_t nnz_blocks;
  int32_t block_size;    /* NB_DOF */
  int32_t ordered_per_block; /* 1: values[k*bs*bs + i*bs + j]; 0: CSR-row order */
  const int64_t* rows;   /* device [n_block_rows+1] */
  const int32_t* columns;/* device [nnz_blocks] */
  double* values;        /* device [nnz_blocks*bs*bs] */
} afem_csr_view;

/* BSRFormat::initialize (femutils/BSRFormat.h:389-409). use_csr_in_linear_system
 * selects the "ordered per row" value layout (values of a scalar row contiguous,
 * as Hypre consumes them) instead of "ordered per block". */
int afem_bsr_create(afem_mesh* mesh, int nb_dof, int use_csr_in_linear_system, afem_bsr** out);
/* BSRFormat::computeSparsity (femutils/BSRFormat.h:749-781): rows are the
 * owned nodes, columns every node sharing an edge (plus the diagonal).  Also
 * builds the row-local incidence table the assembly kernels gather from. */
int afem_bsr_compute_sparsity(afem_bsr* bsr);
/* BSRFormat::assembleBilinear with the P1 Laplacian element of
 * modules/poisson/FemModule.h:139-186, scaled by `coef`, fused with
 * applyConstantSourceToRhs (femutils/ArcaneFemFunctionsGpu.h:401-429) when
 * rhs != NULL: rhs[dof] += sum f*|K|/nv over the cells of own node dof
 * (accumulated, as the reference's doAtomic<Add> at :419-428; device pointer
 * of length n_own_nodes).  Every matrix value of the structure is written (no
 * separate zeroing). */
int afem_bsr_assemble_poisson_p1(afem_bsr* bsr, double coef, double f, double* rhs);
/* RHS modes of the fused source term */
#define AFEM_RHS_ADD 0 /* rhs += source (applyConstantSourceToRhs) */
#define AFEM_RHS_SET 1 /* rhs  = source: the module's rhs_values.fill(0.0) +
                          applyConstantSourceToRhs (modules/poisson/FemModule.cc:163-169) in one pass */
int afem_bsr_assemble_poisson_p1_ex(afem_bsr* bsr, double coef, double f, double* rhs, int rhs_mode);
/* Block-2 P1 elasticity on triangles (modules/elasticity/FemModule.h:112-140),
 * mu2 = 2*mu, lambda as in modules/elasticity/FemModule.cc:130-134. */
int afem_bsr_assemble_elasticity_p1(afem_bsr* bsr, double lambda, double mu2);
/* Block-3 P1 elasticity on tetrahedra (the 3D form of the same bilinear form;
 * no reference module) plus mass_coef * consistent mass (the
 * c0 term of the Newmark / generalized-alpha LHS,
 * modules/elastodynamics/FemModule.cc:259,1285-1340) and, if body_force
 * (3 doubles, host) is given, the vectorial constant source
 * rhs[3n+i] = f_i |K| / 4 on owned nodes (femutils/ArcaneFemFunctionsGpu.h:514-586;
 * rhs: device, 3*n_own; rhs_mode AFEM_RHS_ADD / AFEM_RHS_SET as for the Poisson
 * source). afem_bsr_assemble_elasticity_p1 on a tetrahedral
 * block-3 matrix is this call with mass_coef = 0 and no body force. */
int afem_bsr_assemble_elasticity_p1_ex(afem_bsr* bsr, double lambda, double mu2, double mass_coef,
                                       const double* body_force, double* rhs, int rhs_mode);
int afem_bsr_reset_values(afem_bsr* bsr);                       /* resetMatrixValues */
int afem_bsr_set_value(afem_bsr* bsr, int32_t row, int32_t col, double v); /* BSRMatrix::setValue */
int afem_bsr_get_value(afem_bsr* bsr, int32_t row, int32_t col, double* v); /* BSRMatrix::getValue */
int afem_bsr_view(afem_bsr* bsr, afem_csr_view* view);
/* Structure statistics (for roofline accounting and diagnostics). */
typedef struct afem_bsr_stats {
  int64_t n_incidences;     /* (owned row, incident cell) pairs = entries of the incidence table */
  int64_t inc_table_entries;/* incidence table size including sliced-ELL padding */
  int32_t max_row_len;      /* max non-zero blocks in a row */
  int32_t rows_per_block;   /* rows per assembly wavefront (64: LDS slice tiles; 0: global-memory accumulation variant) */
  int64_t max_seg;          /* max non-zero blocks of one slice (64 rows in processing order) */
  int32_t max_slice_nodes;  /* max distinct nodes one slice couples to (LDS coordinate cache) */
  int32_t max_slice_width;  /* max row length within one slice */
  int64_t n_slices;         /* assembly slices (wavefronts per launch) */
  int32_t brick_order;      /* 1: slices are node bricks of a structured box: 4x4x4 interior bricks
                               (8x8 in 2D), 8x8 tiles of the boundary faces, runs of 32 along the box
                               edges and one slice per corner; 2: the same bricks of
                               a lattice recovered from the coordinates of a mesh given as arrays
                               (any numbering); 0: slices follow a Hilbert-curve order of the node
                               coordinates (plain node order under AFEM_ORDER=node) */
  int32_t uniform_slices;   /* slices whose 64 rows share one strip topology (uniform-control assembly variant) */
  int32_t last_kernel;      /* AFEM_KERNEL_* that ran the last assembly of this matrix */
  int32_t stencil_slices;   /* uniform slices of a compiled-in strip signature (scalar stencil instance) */
  int32_t stencil_sig;      /* that signature's index (-1: none) */
  int64_t shared_strip_slices; /* stencil slices reading their signature's one copy of the per-lane
                                  local-index stream (byte-identical streams: interior bricks) */
  int64_t uniform_instance_slices; /* scalar assembly: uniform slices run by the uniform instance (no
                                      compiled-in signature, not folded into the general list) */
  int64_t general_slices;   /* scalar assembly: slices of the general instance's lists (with the
                               folded uniform ones: a box's edge runs and corners) */
  int32_t cube_lattice;     /* the cell-first cube kernel's view of the mesh (NB_DOF 1 tets): 1 a
                               generator box or z-slab; 2 a Kuhn lattice given as arrays in a natural
                               (lexicographic, any axis order) numbering: the same kernel, no map;
                               3 a Kuhn lattice in any other numbering (canonical maps); 0 none */
  int32_t cube_axes;        /* cube_lattice 2: the numbering's axis order, fastest first, as
                               a0 + 3 a1 + 9 a2 (x + Lx (y + Ly z): 0 + 3 + 18 = 21) */
} afem_bsr_stats;
#define AFEM_KERNEL_NONE 0
#define AFEM_KERNEL_STRIP 1          /* scalar row-strip kernel (uniform + general instances) */
#define AFEM_KERNEL_SLICE_TILE 2     /* scalar incidence-table kernel with the LDS slice tile */
#define AFEM_KERNEL_GLOBAL 3         /* scalar global-memory kernel (no strips, rows beyond the LDS tile) */
#define AFEM_KERNEL_ELAST3_STRIP 4   /* block-3 persistent strip kernel */
#define AFEM_KERNEL_ELAST3_ITEM 5    /* block-3 one-wave-per-item strip kernel */
#define AFEM_KERNEL_ELAST3_GLOBAL 6  /* block-3 global-memory kernel (no strips) */
#define AFEM_KERNEL_ELAST2 7         /* block-2 triangle kernel */
#define AFEM_KERNEL_ELAST3_WG 8      /* block-3 persistent strip kernel, one 3-wave workgroup per slice */
#define AFEM_KERNEL_ELAST3_BIG 9     /* block-3 persistent strip kernel for unstructured meshes (rows <= 32) */
#define AFEM_KERNEL_CUBES 10         /* scalar cell-first cube kernel (generator Kuhn boxes and slabs) */
int afem_bsr_get_stats(afem_bsr* bsr, afem_bsr_stats* stats);
/* Copies the scalar CSR expansion to host in the reference's CSRFormatView
 * layout (BSRMatrix::toCsr, femutils/BSRFormat.h:194-256): rows[n] without
 * sentinel, rows_nb_column[n], columns[nnz], values[nnz] with n = rows*NB_DOF.
 * Any pointer may be NULL; sizes via afem_bsr_get_sizes. */
int afem_bsr_get_sizes(afem_bsr* bsr, int64_t* n_scalar_rows, int64_t* nnz_scalar);
int afem_bsr_export_csr32(afem_bsr* bsr, int32_t* rows, int32_t* rows_nb_column, int32_t* columns, double* values);
/* Device pointers of a structure for a generic element-functor assembly
 * (include/arcanefem_amd_generic.hpp: BSRFormat::assembleBilinear(lambda),
 * femutils/BSRFormat.h:786-837): the mesh's cells and coordinates, the BSR
 * rows / sorted columns / values in the matrix's layout, a device error flag
 * and the context stream (hipStream_t) the kernel is enqueued on.  Valid until
 * the structure is recomputed or destroyed. */
typedef struct afem_assembly_view {
  int64_t n_rows;            /* owned nodes = block rows */
  int64_t n_nodes;           /* local nodes (columns) */
  int64_t n_cells;
  int32_t nb_node_per_cell;
  int32_t block_size;        /* NB_DOF */
  int32_t ordered_per_block; /* value layout, as afem_csr_view */
  int32_t dim;
  const int32_t* cell_node;  /* device [n_cells*nb_node_per_cell] */
  const double* coords;      /* device [n_nodes*3] */
  const int64_t* rows;       /* device [n_rows+1] */
  const int32_t* columns;    /* device [nnz_blocks], sorted per row */
  double* values;            /* device [nnz_blocks*NB_DOF^2] */
  int32_t* error_flag;       /* device, one int: set when an element couples nodes outside the sparsity */
  void* stream;              /* hipStream_t of the structure's context */
} afem_assembly_view;
int afem_bsr_assembly_view(afem_bsr* bsr, afem_assembly_view* view);
/* Cell-unit plan of a structure for generic element functors: what the
 * atomic-free cell kernel of include/arcanefem_amd_generic.hpp
 * (afem::generic::assemble_bilinear) walks.  The reference's
 * BSRFormat<NB_DOF>::assembleBilinear(f) (femutils/BSRFormat.h:786-837,
 * 937-1100, 1105-1111) evaluates f once per cell and scatters with global
 * atomics (or once per (row, cell) without them).  Here one wavefront owns a
 * UNIT -- at most 64 owned rows per layer: a column of fx x fy lattice nodes
 * over a segment of z layers (meshes on a lattice: the generator's boxes and
 * array-fed lattice meshes), else 64/NB_DOF^2-row pieces of the structure's
 * processing-order slices -- and keeps the k x k blocks of its rows in LDS
 * (two layers live).  A unit's cells come in STAGES (stage L: the cells whose
 * highest in-unit vertex lies in layer L; after stage L layer L-1 is
 * complete and is written out): every lane evaluates f for one cell of the
 * stage at a time and adds the rows it owns into LDS.  Entries (one per
 * (unit, cell)): compact (width <= 16): 4 u32 {cell, slots of vertices 0|1,
 * slots of 2|3 (4 bits per vertex b), row positions (8 bits per vertex a:
 * 0x80 valid | layer parity << 6 | lane)}; wide: 4 u32 of 8-bit slots per
 * vertex + 2 u32 {cell, positions}.  Built at the first call (one-time,
 * device), rebuilt with the structure; owned by bsr. */
typedef struct afem_functor_unit {
  int64_t first_stage;       /* index of the unit's first stage (= layer) */
  int32_t n_stages;          /* layers of the unit */
  int32_t flags;             /* 1: rows come in runs of 8 consecutive rows per 8 lanes (coalesced write-back) */
} afem_functor_unit;
typedef struct afem_functor_plan {
  int64_t n_units;
  int64_t n_stages;          /* stages (= layers) over all units */
  int64_t n_entries;         /* (unit, cell) pairs: cell evaluations per assembly */
  int32_t rows_per_layer;    /* lanes that own a row (<= 64) */
  int32_t width;             /* slot stride of the LDS accumulators (max row length) */
  int32_t nbuf;              /* 2: two layers live (lattice columns), 1: single-layer units */
  int32_t wide;              /* entry format: 0 compact, 1 wide */
  int32_t block_size;        /* NB_DOF */
  int32_t nb_node_per_cell;
  int32_t ordered_per_block; /* value layout, as afem_csr_view */
  int32_t lattice;           /* 1: lattice columns, 0: slice pieces */
  const afem_functor_unit* units; /* device [n_units] */
  const int64_t* stage_ptr;  /* device [n_stages+1]: entries of stage s are [stage_ptr[s], stage_ptr[s+1]) */
  const int32_t* layer_rows; /* device [n_stages*rows_per_layer]: row of (stage, lane) or -1 */
  const uint32_t* entries;   /* device, 16 B per entry (see above; 8 B when packed) */
  const uint32_t* entries2;  /* device, wide format: 8 B per entry (cell, positions); else NULL */
  const int64_t* rows;       /* device [n_rows+1] block-row offsets */
  double* values;            /* device, the matrix's values */
  void* stream;              /* hipStream_t of the structure's context */
  /* packed entries (compact plans whose entries repeat few distinct slot /
   * position words, e.g. lattice meshes in a lexicographic numbering): 8 B per
   * entry {cell, pattern}, the pattern's 4 u32 {0, slots 0|1, slots 2|3,
   * positions} in patterns[4 * pattern] -- the compact entry with the cell
   * moved out */
  const uint32_t* patterns;  /* device [n_patterns * 4] when packed, else NULL */
  int64_t n_patterns;
  int32_t packed;            /* 1: entries are 8 B {cell, pattern} */
  int32_t reserved0;
} afem_functor_plan;
int afem_bsr_functor_plan(afem_bsr* bsr, afem_functor_plan* plan);
/* BSRFormat::toLinearSystem with use_csr (femutils/BSRFormat.h:414-430 through
 * BSRMatrix::toCsr, :194-256) in the CALLER's DoF numbering, on the device:
 * dof_of[node*NB_DOF + i] (host, n_nodes*NB_DOF entries: owned and ghost
 * nodes in libafem's numbering) is the caller's DoF local id, n_dof_rows the
 * caller's DoF count.  The CSR has n_dof_rows rows in the CSRFormatView layout
 * (rows without sentinel, rows_nb_column, columns = caller DoF ids in block
 * order; rows of DoFs that are not owned are empty, the isOwn filter of
 * :815, 870), device memory owned by bsr.  dof_of != NULL (re)builds the
 * structure (one time); NULL reuses it.  Every call puts the current values in
 * that order (one gather kernel on the context stream; no copy at all when the
 * map is the identity: values then alias the matrix). */
typedef struct afem_csr32_view {
  int64_t n_rows;
  int64_t nnz;
  const int32_t* rows;           /* device [n_rows] */
  const int32_t* rows_nb_column; /* device [n_rows] */
  const int32_t* columns;        /* device [nnz] */
  double* values;                /* device [nnz] */
  int32_t identity;              /* 1: values alias the matrix's own array */
} afem_csr32_view;
int afem_bsr_to_csr32_mapped(afem_bsr* bsr, const int32_t* dof_of, int64_t n_dof_rows, afem_csr32_view* out);
/* Copies the internal (block) arrays to host. */
int afem_bsr_download(afem_bsr* bsr, int64_t* rows, int32_t* columns, double* values);
/* BSRFormat::toLinearSystem (femutils/BSRFormat.h:414-430): hands the matrix to
 * the linear system as a CSR view (no copy).  The view stays owned by bsr. */
int afem_bsr_to_linear_system(afem_bsr* bsr, afem_ls* ls);
int afem_bsr_destroy(afem_bsr* bsr);

/* ---------------------------------------------------------------- linear system */
#define AFEM_SOLVER_AUTO 0   /* direct below 500 rows on one rank, Jacobi-PCG otherwise
                                (SequentialDoFLinearSystemImpl::solve, femutils/DoFLinearSystem.cc:127-151) */
#define AFEM_SOLVER_PCG 1    /* Jacobi (diagonal) preconditioned CG */
#define AFEM_SOLVER_DIRECT 2 /* dense LU with partial pivoting on the device (one rank, n_rows <= 4096) */

typedef struct afem_solver_opts {
  int32_t method;       /* AFEM_SOLVER_* */
  int32_t max_iter;     /* default 10000 */
  double rtol;          /* stop when sqrt(r.z/r0.z0) <= rtol (default 1e-15, the reference epsilon) */
  double atol;          /* or when ||r||_2 <= atol (default 0 = off) */
  int32_t check_every;  /* iterations between host convergence checks (default 8) */
  int32_t fixed_iterations; /* >0: run exactly this many iterations, no test (benchmarking) */
  int32_t initial_guess;    /* 0: zero (constraint rows lifted to their values, default); 1: start from the
                               current solution vector (free rows; e.g. the previous time step's).  The
                               stopping reference r0.z0 stays the zero guess's: same residual target. */
  int32_t precond_block;    /* 0 or 1: point Jacobi (default); 3: block Jacobi on 3x3 node blocks (NB_DOF = 3
                               systems; constraint rows decoupled from their block mates) */
  int32_t multigrid;        /* 0: off (default); 1: geometric multigrid V-cycle preconditioner (Galerkin coarse
                               operators of the Kuhn-box hierarchy, damped-Jacobi smoothing) on systems from a
                               structured box -- one rank, or its z-slabs over several ranks (one global
                               V-cycle: fine level distributed over the halo, coarse levels replicated) --
                               rebuilt at every solve; 2: built at the first solve
                               and reused while the matrix structure stays the same (time stepping with a
                               constant operator).  Other systems fall back to point Jacobi. */
  int32_t profile_comm;     /* 1: time every halo wait and all-reduce of the PCG loop with HIP events on the
                               context stream (afem_solve_stats.halo_wait_ms / allreduce_ms; diagnostic, adds
                               event records to each iteration); 0: off (default) */
  int32_t amg;              /* 0: off (default); 1: algebraic multigrid V-cycle preconditioner (aggregation AMG
                               built from the CSR on the device: any mesh, one rank), rebuilt at every solve;
                               2: built once and reused while the matrix arrays stay the same.  Where
                               `multigrid` is set and the geometric hierarchy exists, that one is used. */
} afem_solver_opts;

typedef struct afem_solve_stats {
  int32_t iterations;
  int32_t converged;
  double rel_residual;  /* sqrt(r.z / r0.z0) */
  double residual_norm; /* ||b - A x||_2 over all ranks (recurrence residual) */
  double solve_ms;      /* device time of the solve */
  int32_t spmv_kernel;  /* AFEM_SPMV_*: the SpMV the iteration ran */
  /* several ranks (halo attached): the communication of the PCG loop.  With
   * afem_solver_opts.profile_comm the device time the context stream spent
   * waiting for the halo of the search direction after its interior rows (the
   * overlapped split) or in the whole exchange (no split), and in the scalar
   * all-reduces, summed over the iterations; 0 otherwise */
  double halo_wait_ms;
  double allreduce_ms;
  int64_t halo_bytes;   /* bytes this rank sends per halo exchange (8 per shared owned DoF and neighbour) */
  int32_t n_halo;       /* halo exchanges of the loop */
  int32_t n_allreduce;  /* scalar all-reduces of the loop */
  /* the algebraic multigrid hierarchy of the solve (afem_solver_opts.amg; 0 without) */
  int32_t amg_levels;
  int64_t amg_coarse_rows;   /* rows of the coarsest level */
  double amg_complexity;     /* operator complexity: non-zeros of all levels / the matrix's */
  double amg_setup_ms;       /* host time of this solve's hierarchy build (0 when reused; inside solve_ms) */
  /* with afem_solver_opts.profile_comm: device time of the loop's preconditioner
   * applications (multigrid / AMG cycles, HIP events), else 0 */
  double precond_ms;
} afem_solve_stats;
#define AFEM_SPMV_STREAM 0   /* CSR-stream (columns read from the CSR) */
#define AFEM_SPMV_PATTERN 1  /* CSR-stream, interior-stencil rows form their columns */
#define AFEM_SPMV_VECTOR 2   /* 16 lanes per row */
#define AFEM_SPMV_BLOCK 3    /* node-block rows (NB_DOF 2 / 3) */
#define AFEM_SPMV_OTHER 4    /* row-per-thread / no-unroll variants, direct solver */

/* IDoFLinearSystemFactory::createInstance: a linear system over n_rows owned
 * DoFs; n_cols_local >= n_rows counts owned + ghost DoFs (column space of a
 * subdomain). */
int afem_ls_create(afem_ctx* ctx, int64_t n_rows, int64_t n_cols_local, afem_ls** out);
int afem_ls_set_solver_options(afem_ls* ls, const afem_solver_opts* opts);
int afem_ls_get_solver_options(afem_ls* ls, afem_solver_opts* opts);
/* matrixAddValue / matrixSetValue.  With a CSR view set (Hypre semantics,
 * femutils/HypreDoFLinearSystem.cc:148-156) they update the view in place and
 * fail with AFEM_ERR_NOT_FOUND outside the structure.  Without a view they are
 * recorded on the host (Aleph semantics, femutils/AlephDoFLinearSystem.cc:
 * 192-223: adds of 0 skipped, a set overrides every add at solve time) and
 * turned into a device CSR by afem_ls_solve. */
int afem_ls_matrix_add_value(afem_ls* ls, int32_t row, int32_t col, double v);
int afem_ls_matrix_set_value(afem_ls* ls, int32_t row, int32_t col, double v);
/* eliminateRow / eliminateRowColumn (femutils/DoFLinearSystem.h:161-190,
 * semantics of femutils/AlephDoFLinearSystem.cc:501-583), applied at solve. */
int afem_ls_eliminate_row(afem_ls* ls, int32_t row, double v);
int afem_ls_eliminate_row_column(afem_ls* ls, int32_t row, double v);
/* setCSRValues with the reference's CSRFormatView layout: rows[nb_row] (no
 * sentinel; the last row ends at nb_nz), rows_nb_column[nb_row] (may be NULL),
 * columns[nb_nz], values[nb_nz].  The view is non-owning and must stay valid
 * until solve (femutils/DoFLinearSystem.h:251-258).  Device memory: the
 * view is used in place (the BC kernels update its values at solve).  Host
 * memory: structure and values are copied to the device now, matrixAdd/
 * SetValue edit the caller's arrays (and the copy), and afem_ls_solve
 * re-reads the values from the caller's array first, so edits made to the
 * view after this call are seen by the solve; the BCs go into the device copy. */
int afem_ls_set_csr_values(afem_ls* ls, const int32_t* rows, const int32_t* rows_nb_column, const int32_t* columns,
                           double* values, int32_t nb_row, int32_t nb_nz, int mem);
/* setCSRValues for a DEVICE view in the caller's numbering (several
 * subdomains: Arcane interleaves owned and ghost DoFs): index[lid] is the
 * linear system's index of caller DoF lid (owned: [0, n_rows), ghosts:
 * [n_rows, n_cols), -1 none; host, n_index entries).  The owned rows are kept
 * in the linear system's order (structure built here, on the device); the
 * caller's values stay the matrix until solve (re-read there), point updates
 * and afem_ls_apply_boundary_conditions write through to them. */
int afem_ls_set_csr_values_mapped(afem_ls* ls, const int32_t* rows, const int32_t* rows_nb_column,
                                  const int32_t* columns, double* values, int32_t nb_row, int32_t nb_nz,
                                  const int32_t* index, int64_t n_index);
int afem_ls_has_set_csr_values(afem_ls* ls, int* has);
int afem_ls_get_csr_values(afem_ls* ls, afem_csr_view* view);
/* rhsVariable / solutionVariable / getForced{Info,Value} / getElimination{Info,Value}:
 * device arrays of length n_rows (solution: n_cols_local, ghost part filled by
 * the halo after a distributed solve). */
int afem_ls_rhs(afem_ls* ls, double** dptr);
int afem_ls_solution(afem_ls* ls, double** dptr);
int afem_ls_forced_info(afem_ls* ls, uint8_t** dptr);
int afem_ls_forced_value(afem_ls* ls, double** dptr);
int afem_ls_elimination_info(afem_ls* ls, uint8_t** dptr);
int afem_ls_elimination_value(afem_ls* ls, double** dptr);
/* BoundaryConditionsHelpers::applyDirichletToNodeGroupViaPenalty
 * (femutils/ArcaneFemFunctionsGpu.h:434-456): for each owned DoF of the list,
 * forced_info = 1, forced_value = penalty, rhs = penalty * value. */
int afem_ls_dirichlet_penalty(afem_ls* ls, const int32_t* dofs, int64_t n, double value, double penalty, int mem);
/* ...ViaRowElimination (femutils/ArcaneFemFunctionsGpu.h:461-482): elimination_info = 1, value. */
int afem_ls_dirichlet_row_elimination(afem_ls* ls, const int32_t* dofs, int64_t n, double value, int mem);
/* Neumann / traction right-hand side on boundary faces (K15):
 * BoundaryConditions{2D,3D}::applyNeumannToRhs (femutils/ArcaneFemFunctionsGpu.h:612-674,
 * 703-766) and the elasticity traction term (modules/elasticity/FemModule.cc:244-273).
 *   AFEM_NEUMANN_VALUE    rhs[k n]     += value[0] |F| / nf
 *   AFEM_NEUMANN_NORMAL   rhs[k n]     += (value . N) |F| / nf, N the outward unit normal
 *   AFEM_NEUMANN_TRACTION rhs[k n + i] += value[i] |F| / nf, i < nb_dof
 * |F| = edge length (2D, nf = 2 nodes per face) or triangle area (3D, nf = 3);
 * only owned nodes receive a share.  face_nodes[n_faces*nf] are local node ids;
 * face_cells[n_faces] (may be NULL) the cell each face bounds: the normal is
 * oriented away from it, which is what the reference's
 * isSubDomainBoundaryOutside() swap achieves (without it the node order of the
 * face defines the normal).  Arrays in `mem`; rhs: device, nb_dof*n_own_nodes.
 * Accumulated with f64 atomics (summation order not fixed). */
#define AFEM_NEUMANN_VALUE 0
#define AFEM_NEUMANN_NORMAL 1
#define AFEM_NEUMANN_TRACTION 2
int afem_apply_neumann(afem_mesh* mesh, int nb_dof, int mode, const double value[3], int64_t n_faces,
                       const int32_t* face_nodes, const int32_t* face_cells, int mem, double* rhs);
/* _applyRowElimination + _applyForcedValuesToLhs (femutils/HypreDoFLinearSystem.cc:
 * 319-382) on the CSR view; afem_ls_solve calls it, it is exposed so the
 * assembly step can be timed with it. */
int afem_ls_apply_boundary_conditions(afem_ls* ls);
/* clearValues (femutils/HypreDoFLinearSystem.cc:180-187) */
int afem_ls_clear_values(afem_ls* ls);
/* solve: BCs into the CSR, then (SequentialDoFLinearSystemImpl::solve,
 * femutils/DoFLinearSystem.cc:106-164) a direct dense LU below 500 rows or the
 * Jacobi-PCG whose initial guess lifts the constraint rows.
 * With a communicator attached the SpMV exchanges ghost values and the dot
 * products are summed over ranks (RCCL). */
int afem_ls_solve(afem_ls* ls, afem_solve_stats* stats);
/* y[0:n_rows] = A x (x of length n_cols_local, ghost part exchanged first when
 * a communicator is attached).  Device pointers. */
int afem_ls_spmv(afem_ls* ls, const double* x, double* y);
int afem_ls_destroy(afem_ls* ls);

/* ---- time stepping (callers of the path: modules/elastodynamics, modules/passmo) */
/* out = a*x + b*y + c*z on device arrays of n doubles (z may be NULL): the
 * Newmark right-hand side operand c0 U + c3 V + c4 A
 * (modules/elastodynamics/FemModule.cc:842-862 with etam = etak = 0). */
int afem_vec_lincomb(afem_ctx* ctx, int64_t n, double a, const double* x, double b, const double* y, double c,
                     const double* z, double* out);
/* Newmark-beta state update of modules/elastodynamics/FemModule.cc:429-455
 * (_updateVariables) on device arrays: a' = (u_new-u-dt v)/(beta dt^2) -
 * (1-2beta)/(2beta) a, v += dt((1-gamma)a + gamma a'), a = a', u = u_new. */
int afem_newmark_update(afem_ctx* ctx, int64_t n, double dt, double beta, double gamma, const double* u_new, double* u,
                        double* v, double* a);

/* Native Newmark-beta elastodynamics time loop (BASELINE config C5): the
 * callers of the path modules/elastodynamics/FemModule.cc (Newmark constants
 * :255-270, RHS M (c0 U + c3 V + c4 A) + body force :842-862, update
 * :429-455) and modules/passmo/ElastodynamicModule.cc (3D, re-assembly every
 * step on a fixed structure, :469-536).  Per step: fused block-3 re-assembly
 * of c0 M + K and the body force, mass operator (shares the structure),
 * penalty clamp of the fixed nodes' DoFs, Jacobi-PCG (halo + all-reduces over
 * `comm` when given: one ghosted z-slab per rank), device state update.
 * Lame parameters as modules/elasticity/FemModule.cc:132-133. */
typedef struct afem_elastodynamics afem_elastodynamics;
typedef struct afem_newmark_params {
  double E, nu, rho, dt;
  double body_force[3];
  double penalty; /* <= 0: 1e30 (modules/elasticity/Fem.axl:37-41) */
  double gamma;   /* <= 0: 1/2 (scheme 0 only) */
  double beta;    /* <= 0: (gamma + 1/2)^2 / 4 (scheme 0 only) */
  /* Rayleigh damping C = etam M + etak K and the time scheme of
   * modules/elastodynamics/FemModule.cc:222-296: scheme 0 Newmark-beta,
   * 1 generalized-alpha (gamma = 1/2 + alpf - alpm, beta = (gamma + 1/2)^2 / 4).
   * All zero: the undamped Newmark-beta step. */
  double etam, etak;
  double alpm, alpf;
  int32_t scheme;
  int32_t reserved0;
} afem_newmark_params;
/* fixed_nodes: local node ids (in `mem`) whose 3 DoFs are clamped to 0; comm
 * may be NULL (one subdomain). */
int afem_elastodynamics_create(afem_mesh* mesh, afem_comm* comm, const afem_newmark_params* params,
                               const int32_t* fixed_nodes, int64_t n_fixed, int mem, afem_elastodynamics** out);
int afem_elastodynamics_set_solver_options(afem_elastodynamics* dyn, const afem_solver_opts* opts);
int afem_elastodynamics_step(afem_elastodynamics* dyn, afem_solve_stats* stats);
/* Imposed displacements by penalty (passmo's dirichlet-surface-condition /
 * dirichlet-point-condition with enforce-Dirichlet-method Penalty,
 * modules/passmo/ElastodynamicModule.cc:1923-1939): each listed DoF (local id
 * 3*node + component; non-owned ones ignored) gets diagonal = penalty and
 * rhs = value * penalty at every step, and its value is re-applied to the
 * solution before the Newmark update (_doSolve, :2369-2371).  Replaces the
 * previous list (n = 0 clears it); the fixed nodes of afem_elastodynamics_create
 * stay clamped. */
int afem_elastodynamics_set_dirichlet(afem_elastodynamics* dyn, const int32_t* dofs, const double* values, int64_t n,
                                      int mem);
/* Changes dt from the next step on (passmo shortens the step that would
 * overshoot the final time, modules/passmo/ElastodynamicModule.cc:525-530);
 * the Newmark coefficients follow and a reused multigrid hierarchy is rebuilt. */
int afem_elastodynamics_set_time_step(afem_elastodynamics* dyn, double dt);
/* device arrays of 3*n_own_nodes doubles (DoF lid = 3 node + i) */
int afem_elastodynamics_state(afem_elastodynamics* dyn, double** u, double** v, double** a);
/* The step's operators on the device, for checks and callers that post-process
 * (passmo assembles the same c0 M + K on the CPU, ElastodynamicModule.cc:
 * 1389-1793): lhs = the last step's assembled c0 M + K(c1, c2) (block 3,
 * CSR-row order, the clamped DoFs' penalty diagonal included); scalar_rows /
 * scalar_cols = the same values' scalar CSR structure (3 n_block_rows + 1 row
 * offsets, 9 nnz_blocks columns: what the PCG reads); mass_values = the
 * consistent mass M on that structure; c[11] = the step's constants c0 .. c10
 * (modules/elastodynamics/FemModule.cc:255-290).  Any out pointer may be NULL. */
int afem_elastodynamics_operators(afem_elastodynamics* dyn, afem_csr_view* lhs, const int64_t** scalar_rows,
                                  const int32_t** scalar_cols, const double** mass_values, double* c);
/* Per-phase device times of every step while on (HIP events on the context
 * stream; off by default: no events recorded).  Also times the PCG's
 * preconditioner applications (afem_solve_stats.precond_ms). */
int afem_elastodynamics_profile(afem_elastodynamics* dyn, int on);
typedef struct afem_step_timing {
  double assemble_ms;  /* fused block-3 re-assembly of c0 M + K + body force */
  double rhs_ms;       /* RHS operators: lincombs + mass (and damping) SpMVs */
  double bc_ms;        /* penalty lists + the Newmark predictor (the warm start) */
  double solve_ms;     /* the PCG (setup of a new multigrid hierarchy included) */
  double precond_ms;   /* part of solve_ms: the preconditioner applications */
  double update_ms;    /* imposed values + Newmark state update */
  double total_ms;     /* first to last event */
  int32_t iterations;
  int32_t reserved0;
  int64_t nnz_blocks;   /* block non-zeros of the structure */
  int64_t n_incidences; /* (owned row, incident cell) pairs of the structure */
  int64_t n_nodes;      /* local nodes (owned + ghost) */
  int64_t n_own_nodes;
} afem_step_timing;
/* the last profiled step's times (zeros before the first one) */
int afem_elastodynamics_step_timing(afem_elastodynamics* dyn, afem_step_timing* out);
int afem_elastodynamics_destroy(afem_elastodynamics* dyn);

/* ---------------------------------------------------------------- communicator */
#define AFEM_UNIQUE_ID_BYTES 128
/* ncclGetUniqueId on the root rank; the bytes are broadcast by the caller
 * (e.g. torch.distributed) and passed to afem_comm_create on every rank. */
int afem_comm_unique_id(uint8_t id[AFEM_UNIQUE_ID_BYTES]);
int afem_comm_create(afem_ctx* ctx, const uint8_t id[AFEM_UNIQUE_ID_BYTES], int nranks, int rank, afem_comm** out);
/* Host transport: the communicator moves the halo and the dot-product sums
 * through host memory with the caller's callbacks (the reference's
 * IParallelMng::allReduce / sendRecv, or MPI, or torch.distributed gloo) --
 * for hosts where RCCL cannot run (e.g. several ranks on one GPU) and for
 * tests of the distributed path.  Callbacks return 0 on success.
 *   allreduce_sum: in-place sum over all ranks of n doubles.
 *   exchange: for every neighbour i (n_neighbors, in order), send
 *     send_counts[i] doubles (consecutive in `send`) to neighbor_ranks[i] and
 *     receive recv_counts[i] doubles (consecutive in `recv`) from it. */
typedef struct afem_host_transport {
  void* user;
  int (*allreduce_sum)(void* user, double* buf, int64_t n);
  int (*exchange)(void* user, int n_neighbors, const int32_t* neighbor_ranks, const double* send,
                  const int64_t* send_counts, double* recv, const int64_t* recv_counts);
} afem_host_transport;
int afem_comm_create_host(afem_ctx* ctx, int nranks, int rank, const afem_host_transport* transport,
                          afem_comm** out);
/* Host transport only: enable != 0 runs the exchange callback on a worker
 * thread, so the CG's interior SpMV proceeds while the halo is in flight
 * (halo posted after the pack, joined before the boundary rows; the callbacks
 * are then called from that thread, never concurrently with another call on
 * the same communicator).  Default: synchronous.  Enable it only with an
 * exchange callback that may run on a thread other than the caller's: an MPI
 * transport needs at least MPI_THREAD_SERIALIZED, a Python (ctypes) callback
 * takes the GIL on that thread, so the calling thread must not hold the GIL
 * while it waits in the solve (ctypes releases it around foreign calls). */
int afem_comm_host_async(afem_comm* comm, int enable);
int afem_comm_destroy(afem_comm* comm);
/* In-place sum over ranks of n doubles (device pointer) on the context stream. */
int afem_comm_allreduce_sum(afem_comm* comm, double* dbuf, int64_t n);
/* Attach a halo plan (FemDoFsOnNodes::computeSynchronizeInfos equivalent):
 * per neighbour rank, owned DoFs to send and ghost DoFs (ids >= n_rows) to
 * receive, concatenated in neighbour order; counts per neighbour. */
int afem_ls_set_halo(afem_ls* ls, afem_comm* comm, int n_neighbors, const int32_t* neighbor_ranks,
                     const int64_t* send_counts, const int32_t* send_ids, const int64_t* recv_counts,
                     const int32_t* recv_ids);
/* Halo plan of a structured slab mesh (neighbours rank-1 / rank+1); the
 * linear system may carry NB_DOF = n_rows / n_own_nodes DoFs per node (DoF
 * lid = node lid * NB_DOF + i, femutils/FemDoFsOnNodes.cc:79-109). */
int afem_ls_set_halo_structured(afem_ls* ls, afem_comm* comm, afem_mesh* mesh);
/* The same from any mesh that carries a halo plan: a structured slab or an
 * afem_mesh_create_subdomain subdomain (NB_DOF-aware as above). */
int afem_ls_set_halo_mesh(afem_ls* ls, afem_comm* comm, afem_mesh* mesh);
/* Host-only (no GPU needed): the halo plan of a structured slab mesh, i.e.
 * the ghost synchronisation lists FemDoFsOnNodes::computeSynchronizeInfos
 * builds (femutils/FemDoFsOnNodes.cc:125-126).  Neighbours are rank-1 and
 * rank+1; *n_neighbors receives 0..2; counts per neighbour; pass NULL id
 * arrays to query the counts. */
int afem_structured_halo_plan(int dim, int n, int nz, int nranks, int rank, int* n_neighbors,
                              int32_t* neighbor_ranks, int64_t* send_counts, int64_t* recv_counts, int32_t* send_ids,
                              int32_t* recv_ids);
/* m_u.synchronize(): owner -> ghost copy of a length-n_cols_local device vector. */
int afem_ls_synchronize(afem_ls* ls, double* x);

#ifdef __cplusplus
}
#endif
#endif /* ARCANEFEM_AMD_H */
