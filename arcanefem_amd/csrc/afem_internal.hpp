// Internal declarations of the MI355X FEM assembly + CG library (libafem.so).
// Host side is C++17; kernels are hand-written HIP for gfx950 (CDNA4,
// wave64).  See DESIGN.md for the data layout and the roofline of each kernel.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/arcanefem_amd.h"

namespace afem {

// Value and RHS stores of the row-strip / block-3 assembly kernels: plain by
// default.  Non-temporal stores (-DAFEM_NT_STORES=1) pay off for long
// contiguous runs (the cube kernel's complete-layer flush: 0.520 -> 0.478 ms
// at C2, its V bit 32) but not for these kernels' row-wise write-backs: the
// unstructured leg 0.246 -> 0.262 ms, C3 unchanged (r05h, tools/ab_lib.py).
#ifndef AFEM_NT_STORES
#define AFEM_NT_STORES 0
#endif
template <class T>
__device__ __forceinline__ void st_out(T* p, T v)
{
#if AFEM_NT_STORES
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}


struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

[[noreturn]] void throw_hip(hipError_t e, const char* expr, const char* file, int line);

// kernel-variant knob `name` (AFEM_*): afem_set_variant's value, else the
// environment's at first lookup, else nullptr (the default variant)
const char* variant(const char* name);
void set_variant(const char* name, const char* value);

#define AFEM_HIP(x)                                              \
  do {                                                           \
    hipError_t e_ = (x);                                         \
    if (e_ != hipSuccess) ::afem::throw_hip(e_, #x, __FILE__, __LINE__); \
  } while (0)

#define AFEM_REQUIRE(cond, code, msg)                 \
  do {                                                \
    if (!(cond)) throw ::afem::Error((code), (msg));  \
  } while (0)

// Launch-error check right after a kernel launch (asynchronous faults surface
// at the next synchronising call).
#define AFEM_LAUNCHED() AFEM_HIP(hipGetLastError())

constexpr int kWave = 64;

// ------------------------------------------------------------------ device buffer
template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) { reset(); p = o.p; n = o.n; o.p = nullptr; o.n = 0; }
    return *this;
  }
  ~DevBuf() { reset(); }
  void alloc(size_t count) {
    reset();
    if (count) AFEM_HIP(hipMalloc(reinterpret_cast<void**>(&p), count * sizeof(T)));
    n = count;
  }
  void reset() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  size_t bytes() const { return n * sizeof(T); }
};

// ------------------------------------------------------------------ context
struct Ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::vector<hipEvent_t> pool;  // AFEM_EVENT_SLOTS, created lazily
  // side stream for a small kernel that runs beside a large one (fork/join
  // through two events on the context stream), created lazily
  hipStream_t aux = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipStream_t side()
  {
    if (!aux) {
      AFEM_HIP(hipStreamCreateWithFlags(&aux, hipStreamNonBlocking));
      AFEM_HIP(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
      AFEM_HIP(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
    }
    return aux;
  }
  int n_cu = 256;
  void set_device() const { AFEM_HIP(hipSetDevice(device)); }
  void sync() const { AFEM_HIP(hipStreamSynchronize(stream)); }
};

// ------------------------------------------------------------------ mesh
struct StructuredInfo {
  bool valid = false;
  int dim = 3, n = 0, nz = 0, nranks = 1, rank = 0;
  int64_t lx = 0, ly = 0;   // 3D node counts along x / y when they differ from n + 1 (a relabeled lattice)
  int64_t L = 0;            // nodes per layer
  int k0 = 0, k1 = 0;       // owned node layers [k0,k1)
  int ghost_lo = -1, ghost_hi = -1;  // ghost layers (or -1)
  double jitter = 0.0;
  uint64_t seed = 0;
};

// Subdomain of a partitioned general mesh (partition.cpp): local numbering
// (owned nodes first, then ghosts; l2g = global node ids), local cells
// (global ids) and their local connectivity, halo lists per neighbour rank
// (local node ids; send = owned nodes, receive = ghosts).
struct SubdomainPlan {
  bool valid = false;
  int nranks = 1, rank = 0;
  int64_t n_own = 0;
  std::vector<int64_t> l2g, cells;
  std::vector<int32_t> cell_node;
  std::vector<int> nbr;
  std::vector<int64_t> send_cnt, recv_cnt;
  std::vector<int32_t> send_ids, recv_ids;
};
void partition_rcb(int dim, int64_t n, const double* xyz, int nparts, int32_t* part);
void subdomain_plan(int nv, int64_t n_nodes, int64_t n_cells, const int32_t* cell_node, const int32_t* part,
                    int nranks, int rank, SubdomainPlan& P);

struct Mesh {
  Ctx* ctx = nullptr;
  int dim = 3;
  int nv = 4;
  int64_t n_nodes = 0, n_own = 0, n_cells = 0;
  DevBuf<int32_t> cell_node;  // [n_cells*nv]
  DevBuf<double> coords;      // [n_nodes*3]  AoS x,y,z (VariableNodeReal3 layout)
  StructuredInfo st;
  SubdomainPlan part;  // meshes from afem_mesh_create_subdomain
};

// ------------------------------------------------------------------ sparsity
// Per-slice record of the strip assembly, one 32-B scalar load per slice
// (in the order of the slice lists the kernel walks).
struct alignas(16) SliceRec {
  uint32_t sl;         // slice id (positions 64*sl .. 64*sl+63)
  uint32_t lidx_off;   // lidx_ptr[sl]
  uint32_t strip_off;  // strip_ptr[sl] / 1024
  uint32_t snode_off;  // snode_ptr[sl]
  uint32_t meta;       // slice nodes | width (max row length) << 16 | strip steps << 24
  uint32_t sig;        // stencil list: index of the slice's compiled-in strip signature (else 0)
  uint64_t pat;        // uniform slices: shift/swap bits
};
static_assert(sizeof(SliceRec) == 32, "SliceRec is one s_load_dwordx8");

// Strip signature of a stencil instance (assembly.hip k_assemble_stencil): the
// steps (2 priming + cells), row length, diagonal slot, shift/swap bits and the
// 32 step bytes of the uniform slot stream (k_strip_classify's layout).
struct StencilSig {
  int nsteps, w, dslot;
  uint64_t pat;
  uint8_t slot[32];
};
// index of the compiled-in stencil signature a uniform slice matches, or -1
int stencil_match(uint64_t pat, int nsteps, int w, const uint8_t* slot32);

// Scalar (node-node) structure shared by every NB_DOF: rows = owned nodes.
struct Structure {
  int64_t n_rows = 0, n_cols = 0, nnz = 0;
  DevBuf<int64_t> row_ptr;  // [n_rows+1]
  DevBuf<int32_t> cols;     // [nnz], sorted ascending per row
  // Assembly processing order: slice s (one wavefront) processes the rows
  // perm[64*s + lane] (-1 = idle lane).  Structured boxes use 4x4x4 (3D) /
  // 8x8 (2D) node bricks, so a slice's rows share most neighbours; other
  // meshes use the node order.  The matrix itself stays in node order.
  DevBuf<int32_t> perm;  // [n_slices*64]
  bool brick_order = false;
  bool lattice = false;  // brick order of a lattice recovered from the coordinates (array-fed mesh)
  // Lanes [j*run, (j+1)*run) of a slice hold consecutive rows (an x-run of a
  // brick, or the whole slice in node order), idle lanes only at the end of
  // a run: their value segments are one contiguous range.
  int run = 64;
  // Row-local incidence table, sliced ELLPACK with C = 64 (one wavefront):
  // entry (slice s, k, lane) at inc_slice_ptr[s] + (k/4)*256 + lane*4 + k%4 describes the
  // k-th cell incident to row perm[64*s+lane] as the row-slots of the cell's
  // other nodes (one byte each) and the row's diagonal slot in the top byte.
  DevBuf<uint32_t> inc;
  DevBuf<int64_t> inc_slice_ptr;  // [n_slices+1]
  DevBuf<int32_t> inc_slice_k;    // [n_slices] max incidences in the slice
  int64_t inc_pad_off = 0;        // 256 padding entries at the end (slices without incidences)
  // Per slice: the sorted unique nodes its rows couple to (snode, the
  // coordinate cache the assembly stages in LDS) and, for every (slot t,
  // lane), the index of column cols[row_ptr[row]+t] in that list:
  // lidx[lidx_ptr[s] + 64*t + lane] (0 past the row's end).
  DevBuf<int32_t> slice_w;     // [n_slices] max row length in the slice
  DevBuf<int64_t> lidx_ptr;    // [n_slices+1] = 64 * prefix sum of slice_w
  DevBuf<uint16_t> lidx;
  DevBuf<int64_t> snode_ptr;   // [n_slices+1]
  DevBuf<int32_t> snode;
  int max_slice_nodes = 0, max_slice_w = 0, max_slice_k = 0;
  // Row strips (sparsity.hip, "row strips"): per slice, 16-step chunks of one
  // byte per step per lane at strip_ptr[s] + chunk*1024 + lane*16 + step%16;
  // dslot = diagonal slot of each position's row.
  bool strip_ok = false;
  int max_strip_c = 0;
  DevBuf<uint8_t> strip;
  DevBuf<uint8_t> strip_u;  // per step byte: local index of its node in the slice's node list (u8)
  DevBuf<int64_t> strip_ptr;
  DevBuf<int32_t> strip_c;  // 16-step chunks per slice
  DevBuf<int32_t> strip_n;  // steps per slice (longest row stream)
  DevBuf<uint8_t> dslot;
  // Slices whose 64 rows share one strip topology (one strip, same length,
  // same shift/swap bits spat[s]) run the uniform-control assembly variant;
  // rec_u / rec_m list the uniform / other slices in processing order.
  DevBuf<uint64_t> spat;
  DevBuf<uint8_t> uslot;  // uniform list, in list order: the 32 common step bytes of each slice (scalar stream)
  DevBuf<SliceRec> rec_u, rec_m, rec_all;  // uniform / other / every slice, in processing order
  int64_t n_uni = 0, n_mix = 0;
  // the scalar kernel's split of the other (general-instance) slices: small
  // = at most 16 slots, 32 steps and kSmallSliceNodes nodes (the compact LDS
  // tile, higher occupancy), big = the rest
  DevBuf<SliceRec> rec_ms, rec_mb;
  int64_t n_ms = 0, n_mb = 0;
  // the compact list's first n_msl slices have <= 256 nodes: the instance that
  // reads each step's node from the local-index stream (UMODE 3) runs them
  int64_t n_msl = 0;
  int msl_nodes = 0;
  int ms_nodes = 0, mb_nodes = 0, mb_w = 0;
  int u_nodes = 0, u_w = 0;  // maxima over the uniform list (its LDS tile)
  // stencil split of the uniform list (scalar assembly): the slices of any
  // compiled-in signature (rec_k, SliceRec::sig; sig_k = the most frequent
  // one, -1 if none) and the other uniform slices (rec_ur + their slot
  // streams urslot); rec_u stays whole (block-3 uses it)
  DevBuf<SliceRec> rec_k, rec_ur;
  DevBuf<uint8_t> urslot;
  // block-3 split of the uniform list: signature-0 slices (rec_k0) and the rest
  // (rec_u1 + their slot streams u1slot)
  DevBuf<SliceRec> rec_k0, rec_u1;
  DevBuf<uint8_t> u1slot;
  int64_t n_k0 = 0, n_u1 = 0;
  int64_t n_k = 0, n_ur = 0;
  int sig_k = -1, k_nodes = 0, ur_nodes = 0, ur_w = 0;
  int64_t n_strip_shared = 0;  // stencil slices reading their signature's shared strip_u copy
  bool rec_ok = false;                     // offsets fit the 32-bit record fields
  DevBuf<int64_t> pos_rb;                  // [n_slices*64] row_ptr of each position's row (0: idle)
  DevBuf<uint32_t> pos_dl;                 // [n_slices*64] diagonal slot | row length << 8
  DevBuf<unsigned long long> tickets;  // dynamic slice claiming (assembly): a ring of per-assembly counter slots
  int64_t ticket_gen = 0;              // assemblies since the ring was last zeroed (assembly.hip next_tickets)
  int64_t n_slices = 0;
  int64_t n_incidences = 0;  // real (non-padding) entries
  int max_row_len = 0;
  int64_t max_wave_seg = 0;  // max nnz of one slice
  DevBuf<int64_t> diag_pos;  // [n_rows] position of the diagonal in cols
  // canonical lattice structure (array-fed lattice meshes in any numbering,
  // NB_DOF 1; sparsity.hip canonical_lattice): the assembly metadata (slices,
  // strips, slot streams, node lists) is built in the lattice's own numbering,
  // where a row's slots follow the generator box's column order and the
  // compiled-in strip signatures match; cperm[16 p + t] is the position in the
  // row's (id-sorted) columns of the row's canonical slot t at processing
  // position p.  The strip / stencil kernels write through it.
  bool canon = false;
  DevBuf<uint8_t> cperm;
  // canonical lattice of Kuhn cubes (every cell one of the 6 Kuhn tets of its
  // cube): the cube kernel runs on it (cubes.hip).  Per lattice node i: the
  // caller's node, its row's first value, and the position in that row of
  // canonical slot t (4 bits each)
  bool cube_ok = false;
  int64_t cube_L[3] = { 0, 0, 0 };
  // a lattice of Kuhn cubes handed over as arrays in a NATURAL numbering:
  // node id = lexicographic lattice index with the axes taken in the order
  // cube_axes (fastest first; x + Lx (y + Ly z) is {0, 1, 2}), every node
  // owned -- the generator's layout up to the axis order, so the cube
  // kernel's plain instance runs on it (nat_L: the lattice's node counts in
  // that axis order; no maps)
  bool cube_natural = false;
  int nat_axes[3] = { 0, 1, 2 };
  int64_t nat_L[3] = { 0, 0, 0 };
  DevBuf<int32_t> cube_phys;
  DevBuf<int64_t> cube_rb;
  DevBuf<uint64_t> cube_slot;
  // the staged canonical path (cubes.hip, built at its first use): per CALLER
  // row its lattice index and, per position p of its columns, the Kuhn offset
  // o (0..14) whose value goes there (4 bits each)
  DevBuf<int32_t> cube_lat;
  DevBuf<uint64_t> cube_pinv;
};

struct LinearSystem;

// Cell-unit plan of a structure for generic element functors
// (functor_plan.hip; the kernel is the header template
// include/arcanefem_amd_generic.hpp k_assemble_units): units of at most 64
// rows per layer -- lattice columns of fx x fy nodes cut into z segments of
// zs layers (every cell spans at most two consecutive layers), or rl-row
// pieces of the processing-order slices (one layer) -- and, per (unit, layer)
// "stage", the cells whose highest in-unit vertex lies in that layer, each
// with the unit-local row position and the row slots of its vertices.
struct FunctorPlan {
  bool valid = false;
  int nb_dof = 0;
  int rl = 64, w = 0, nbuf = 1, wide = 0, lattice = 0;
  int fx = 0, fy = 0, zs = 1;
  int64_t n_units = 0, n_stages = 0, n_entries = 0, n_coalesced = 0;
  DevBuf<afem_functor_unit> units;
  DevBuf<int64_t> stage_ptr;   // [n_stages + 1]
  DevBuf<int32_t> layer_rows;  // [n_stages * rl]
  DevBuf<uint32_t> ent, ent2;  // compact: 4 u32 per entry; wide: 4 u32 slots + 2 u32 (cell, pos); packed: 2 u32
  int packed = 0;
  int64_t n_patterns = 0;
  DevBuf<uint32_t> patterns;   // packed: 4 u32 per pattern {0, slots 0|1, slots 2|3, positions}
};
void functor_plan_build(struct Bsr& b);

// BSRFormat::toLinearSystem in the caller's DoF numbering (handover.hip):
// the scalar CSR (int32, CSRFormatView layout) and the value gather index
struct HandOver {
  bool valid = false, identity = false;
  int64_t n_rows = 0, nnz = 0;
  DevBuf<int32_t> rows, rnc, cols;
  DevBuf<int64_t> src;  // value index in the BSR values (not kept when identity)
  DevBuf<double> vals;
};

struct Bsr {
  Mesh* mesh = nullptr;
  int nb_dof = 1;
  bool order_per_block = true;  // false: CSR row order (use_csr_in_linear_system)
  bool has_sparsity = false;
  Structure s;
  DevBuf<double> values;       // [nnz * nb_dof^2]
  int last_kernel = 0;         // AFEM_KERNEL_* of the last assembly launch (afem_bsr_stats)
  // scalar CSR expansion for NB_DOF>1 (built on demand)
  DevBuf<int64_t> csr_rows;
  DevBuf<int32_t> csr_cols;
  DevBuf<double> csr_vals;  // per-block layout permuted to CSR order
  DevBuf<int32_t> gen_flag;  // error flag of the generic element-functor assembly (afem_bsr_assembly_view)
  FunctorPlan fplan;         // cell-unit plan of the generic assembly (built at its first use)
  HandOver hand;             // toLinearSystem in the caller's numbering (afem_bsr_to_csr32_mapped)
  DevBuf<double> cube_stage; // staged canonical cube path: one 128-B line per lattice row (cubes.hip)
};
void bsr_csr32_mapped_build(Bsr& b, const int32_t* dof_of_host, int64_t n_dof_rows);
double* bsr_csr32_mapped_values(Bsr& b);  // the values in the mapped CSR order (gathered, or aliased)

// ------------------------------------------------------------------ communicator / halo
struct Comm;
struct Halo {
  Comm* comm = nullptr;
  std::vector<int> nbr;
  std::vector<int64_t> send_cnt, recv_cnt, send_off, recv_off;
  DevBuf<int32_t> send_ids, recv_ids;
  DevBuf<double> send_buf, recv_buf;
  int64_t n_send = 0, n_recv = 0;
  // split exchange (halo_begin / halo_end): the RCCL send/recv run on their
  // own stream while the context stream computes (created lazily)
  hipStream_t cs = nullptr;
  hipEvent_t ev_packed = nullptr, ev_done = nullptr;
  // asynchronous host transport (afem_comm_host_async): the caller's exchange
  // callback runs on `worker` between halo_begin and halo_end, on the pinned
  // staging buffer hpin (send part, then receive part)
  double* hpin = nullptr;
  size_t hpin_n = 0;
  std::thread worker;
  int worker_rc = 0;
  Halo() = default;
  Halo(const Halo&) = delete;
  Halo& operator=(const Halo&) = delete;
  ~Halo()
  {
    if (worker.joinable()) worker.join();
    if (hpin) (void)hipHostFree(hpin);
    if (ev_packed) (void)hipEventDestroy(ev_packed);
    if (ev_done) (void)hipEventDestroy(ev_done);
    if (cs) (void)hipStreamDestroy(cs);
  }
};

void halo_exchange(Halo& h, Ctx& ctx, double* x);
// halo_exchange in two halves: begin packs and posts the transfers (RCCL: on
// the halo's stream, returns at once; host transport: the whole exchange),
// end makes the context stream wait for them and scatters the ghosts
void halo_begin(Halo& h, Ctx& ctx, double* x);
void halo_end(Halo& h, Ctx& ctx, double* x);
void comm_allreduce(Comm* c, Ctx& ctx, double* d, int64_t n);
bool comm_is_host(Comm* c);  // host-transport communicator
bool comm_self_loop();  // AFEM_COMM_SELF=1: one-rank collectives run anyway (comm.hip)
void comm_set_host_async(Comm* c, bool on);  // host transport: exchange on a worker thread (halo_begin/end)

// ------------------------------------------------------------------ linear system
struct Multigrid;
struct MgDeleter {
  void operator()(Multigrid* m) const;
};
struct Amg;
struct AmgDeleter {
  void operator()(Amg* a) const;
};
struct LinearSystem {
  Ctx* ctx = nullptr;
  std::vector<hipEvent_t> prof_ev;  // afem_solver_opts.profile_comm: event pool of the PCG loop's timings
  int64_t n_rows = 0, n_cols = 0;
  afem_solver_opts opts{};
  DevBuf<double> rhs, sol;
  DevBuf<uint8_t> forced_info, elim_info;
  DevBuf<double> forced_value, elim_value;
  // CSR view (device)
  bool has_csr = false;
  int64_t csr_n = 0, csr_nnz = 0;
  const int64_t* csr_rows = nullptr;
  const int64_t* csr_diag = nullptr;  // diagonal positions when the view is a BSRFormat's own CSR (NB_DOF 1)
  const int32_t* csr_cols = nullptr;
  double* csr_vals = nullptr;
  // node-row structure of a view that came from a BSRFormat with NB_DOF = blk_k
  // (2 or 3; 0: none): the SpMV's column source (k_spmv_blk)
  int blk_k = 0;
  int64_t blk_n = 0;
  const int64_t* blk_rows = nullptr;
  const int32_t* blk_cols = nullptr;
  DevBuf<int64_t> own_rows;   // when the view came in the reference int32 layout
  DevBuf<int32_t> own_cols;
  DevBuf<double> own_vals;    // host-uploaded or COO-built matrix
  // setCSRValues in the caller's numbering (afem_ls_set_csr_values_mapped):
  // the caller's device values stay the matrix (gathered into own_vals at
  // solve, point updates and the BC pass written back through mv_src)
  double* mv_vals = nullptr;
  DevBuf<int64_t> mv_src;
  // setCSRValues on HOST memory: the caller's arrays stay the matrix until the
  // solve (femutils/DoFLinearSystem.h:251-258) -- point updates edit them and
  // afem_ls_solve re-reads the values (own_vals is the device copy)
  const int32_t* hv_rows = nullptr;
  const int32_t* hv_cols = nullptr;
  double* hv_vals = nullptr;
  // the CSR was rebuilt from the host COO maps (matrixAddValue without a
  // view): later adds/sets go to the maps again; any other CSR view (device,
  // host-uploaded, BSR) is updated in place
  bool csr_from_coo = false;
  // host COO (Aleph semantics)
  std::map<std::pair<int32_t, int32_t>, double> add_map, set_map;
  std::map<int32_t, std::pair<uint8_t, double>> host_elim;
  // solver work
  DevBuf<double> r, z, p, q, dinv, partial, scal;
  mutable DevBuf<uint8_t> pat_flag;  // rows whose columns follow the dominant offset pattern (pattern SpMV)
  mutable DevBuf<int32_t> pat_smp;   // the pattern detection's row samples
  mutable DevBuf<unsigned long long> pat_cnt;
  DevBuf<double> x0;      // the caller's initial guess (opts.initial_guess = 1)
  DevBuf<double> binv;    // block-Jacobi 3: inverse node blocks [n/3][9]
  DevBuf<int32_t> blist;  // multi-rank CG: SpMV row blocks, interior ones first
  int64_t blist_nint = 0;
  uint64_t blist_key = 0;
  DevBuf<double> dense;  // direct solver: augmented n x (n+1) matrix
  DevBuf<uint8_t> cons;  // constraint-row flags of the stopping test
  double* pinned = nullptr;
  std::unique_ptr<Halo> halo;
  // structured Kuhn box on one rank (BSR from Mesh.structured): the geometric
  // multigrid preconditioner's fine grid (multigrid.hip); mg_k = NB_DOF, 0: none
  int mg_k = 0, mg_nx = 0, mg_nz = 0;  // the OWNED box: (nx+1)^2 (nz+1) nodes in lexicographic local ids
  // a ghosted subdomain (slab of a multi-rank system): the preconditioner is a
  // local V-cycle on the owned block (ghost columns dropped: block Jacobi over
  // the ranks, no communication), on a box padded by one decoupled layer when
  // the owned cell count in z is odd
  bool mg_multi = false;
  // the slab's place in the global box (z-slabs of Mesh.structured): global
  // cells in z, first owned node layer, whether a ghost layer below exists
  // (local numbering: owned layers, then the ghost layer below, then above).
  // With an even global box the preconditioner is ONE global V-cycle: the fine
  // level distributed (halo exchanges), the coarse levels replicated on every
  // rank (multigrid.hip); AFEM_MG_MULTI=block keeps the block-Jacobi V-cycles
  int mg_nzg = 0, mg_k0 = 0;
  bool mg_glo = false;
  std::unique_ptr<Multigrid, MgDeleter> mg;
  std::unique_ptr<Amg, AmgDeleter> amg;  // algebraic multigrid (amg.hip, afem_solver_opts.amg)
  std::shared_ptr<void> spmv_plan;       // the current solve's SpMV plan (linear_system.hip SpmvPlan)
};

// ------------------------------------------------------------------ kernels (host launchers)
void exclusive_scan_i64(Ctx& ctx, const int64_t* in, int64_t* out, int64_t n, DevBuf<int64_t>* tmp_pool = nullptr);
void exclusive_scan_i32_to_i64(Ctx& ctx, const int32_t* in, int64_t* out, int64_t n);
int64_t read_i64(Ctx& ctx, const int64_t* d);
void device_minmax_i32(Ctx& ctx, const int32_t* a, int64_t n, int32_t* lo, int32_t* hi);

// nb_dof = 1: a lattice mesh in a non-generator numbering gets the canonical
// lattice structure (Structure::canon) when its strips match the compiled-in
// signatures there
void build_structure(Mesh& m, Structure& s, int nb_dof = 0);
// node -> incident-cell lists of the owned nodes (sorted by cell id); returns the entry count
int64_t node_cell_adjacency(Ctx& ctx, const Mesh& m, int64_t n_rows, DevBuf<int64_t>& nc_ptr, DevBuf<int32_t>& nc);
// per-axis layer index of every owned node when they sit on a (jittered) lattice (sparsity.hip)
bool lattice_coords(Ctx& ctx, const Mesh& m, int64_t n_rows, DevBuf<int32_t> layer[3], int64_t L[3]);
// rhs_add: 1 accumulate into rhs (applyConstantSourceToRhs), 0 overwrite
void assemble_scalar(Bsr& b, double coef, double f, double* rhs, int rhs_add);
// the cell-first cube kernel on generator boxes / slabs (cubes.hip); false: not applicable
bool assemble_cubes(Bsr& b, double coef, double f, double* rhs, int rhs_add);
void assemble_elasticity_tri(Bsr& b, double lambda, double mu2);
void assemble_elasticity_tet(Bsr& b, double lambda, double mu2, double c0, const double* f, double* rhs, int rhs_add);
void apply_neumann(Mesh& m, int k, int mode, const double* v, int64_t n_faces, const int32_t* face_nodes,
                   const int32_t* face_cells, int mem, double* rhs);
bool assembly_uses_lds(const Bsr& b);  // slice tile fits the LDS budget

// geometric multigrid preconditioner (multigrid.hip)
bool mg_available(const LinearSystem& ls);
void mg_setup(LinearSystem& ls);                              // (re)build the hierarchy from the current matrix
void mg_apply(LinearSystem& ls, const double* r, double* z);  // z = M^-1 r (one V-cycle)
int mg_levels(const LinearSystem& ls);
// node-block SpMV with an epilogue (linear_system.hip): epi 0: y = A x; 1: y = x + omega dinv (b - A x)
// (a damped-Jacobi sweep); 2: y = b - A x.  NB_DOF k = 1, 2 or 3, values in BSRFormat's CSR order.
void spmv_blk_epi(Ctx& ctx, int k, int epi, int64_t n_brows, const int64_t* bp, const int32_t* bc, const double* vals,
                  const double* x, double* y, const double* b, const double* dinv, double omega);
// the block-3 product on the private fp32 layout (k_spmv_blk3f) and that layout from the CSR order
void spmv_blk3f_epi(Ctx& ctx, int epi, int64_t n_brows, const int64_t* bp, const int32_t* bc, const float* vf,
                    const double* x, double* y, const double* b, const double* dinv, double omega,
                    const uint8_t* cons = nullptr, const double* rin = nullptr, const double* dfix = nullptr);
void blk3_to_f32(Ctx& ctx, int64_t n_brows, const int64_t* bp, const double* vals, float* vf);
void ls_apply_bcs(LinearSystem& ls);
void ls_set_csr_mapped(LinearSystem& ls, const int32_t* rows, const int32_t* columns, double* values, int32_t nb_row,
                       int32_t nnz, const int32_t* index_host, int64_t n_index);
void ls_mapped_gather(LinearSystem& ls);
void ls_mapped_scatter_back(LinearSystem& ls);
void ls_mapped_point_update(LinearSystem& ls, int32_t row, int32_t col, double v, bool set);
void ls_solve(LinearSystem& ls, afem_solve_stats* st);
void ls_spmv(LinearSystem& ls, const double* x, double* y);
void ls_spmv_planned(LinearSystem& ls, const double* x, double* y);
// algebraic multigrid preconditioner (amg.hip)
bool amg_available(const LinearSystem& ls);
bool amg_nonlinear(const LinearSystem& ls);  // a K-cycle level: the preconditioner depends on r
bool amg_setup(LinearSystem& ls);  // false: the amg-reuse hierarchy was kept
void amg_apply(LinearSystem& ls, const double* r, double* z);
void amg_stats(const LinearSystem& ls, int32_t* levels, int64_t* coarse_rows, double* complexity);
void ls_build_from_host_coo(LinearSystem& ls);
void ls_point_update(LinearSystem& ls, int32_t row, int32_t col, double v, bool set);
// kind 0 penalty, 1 row elimination, 2 row+column elimination of the listed DoFs
// (owned ones); dvalues (device, one per id; ids in device memory) or the
// common value
void ls_set_list(LinearSystem& ls, const int32_t* ids, int64_t n, int mem, int kind, double value, double penalty,
                 const double* dvalues = nullptr);

void mesh_structured(Ctx& ctx, Mesh& m, int dim, int n, int nz, double jitter, uint64_t seed, int nranks, int rank);
void mesh_structured_bottom(Mesh& m, std::vector<int32_t>& ids);
void mesh_local_to_global(Mesh& m, int64_t* host_out);
void structured_halo_lists(int dim, int n, int nz, int nranks, int rank, std::vector<int>& nbr,
                           std::vector<int64_t>& send_cnt, std::vector<int64_t>& recv_cnt,
                           std::vector<int32_t>& send_ids, std::vector<int32_t>& recv_ids);

void expand_dof_lists(int k, std::vector<int64_t>& sc, std::vector<int64_t>& rc, std::vector<int32_t>& si,
                      std::vector<int32_t>& ri);

// op: 0 get, 1 set, 2 add on the (scalar DoF row, scalar DoF col) entry of a BSR
// matrix; returns false when the entry is not in the structure.
bool bsr_point(Bsr& b, int32_t row, int32_t col, int op, double v, double* out);
// Scalar CSR expansion of an NB_DOF>1 matrix (BSRMatrix::toCsr,
// femutils/BSRFormat.h:194-256) into b.csr_rows/b.csr_cols; values: the
// per-row layout is already CSR order, the per-block one is permuted into
// `vals_out` (device, nnz*k^2).
void bsr_expand_scalar(Bsr& b, double* vals_out);

// ------------------------------------------------------------------ time stepping (elastodynamics.cpp)
struct Elastodynamics {
  Mesh* mesh = nullptr;
  Ctx* ctx = nullptr;
  Comm* comm = nullptr;
  afem_newmark_params p{};
  double lambda = 0, mu2 = 0, gamma = 0.5, beta = 0.25;
  double c[11] = {};      // modules/elastodynamics/FemModule.cc:255-290 c0 .. c10
  bool damped = false;    // a stiffness term on the RHS (etak != 0 or alpf != 0)
  Bsr K;                  // block-3, per-row (CSR) layout: values = c0 M + K(c1, c2)
  DevBuf<double> mvals;   // consistent mass on K's structure (CSR order)
  DevBuf<double> klvals, kmvals;  // damped: K(lambda = 1, 2 mu = 0) and K(0, 1) on K's structure
  LinearSystem ls, lsm;   // the solve, and the mass operator's SpMV
  LinearSystem lsl, lsu;  // damped: the SpMVs of klvals / kmvals
  DevBuf<double> U, V, A, W, MW;
  DevBuf<int32_t> fixed;  // clamped DoFs
  DevBuf<int32_t> imp_ids;  // imposed displacements (afem_elastodynamics_set_dirichlet): owned DoFs
  DevBuf<double> imp_vals;  //   and their values
  int64_t n = 0, n_cols = 0;
  afem_solve_stats last{};
  // afem_elastodynamics_profile: per-phase events of every step
  bool profile = false;
  hipEvent_t ev[6] = {};
  afem_step_timing timing{};
};
Elastodynamics* dyn_create(Mesh* mesh, Comm* comm, const afem_newmark_params* prm, const int32_t* fixed_nodes,
                           int64_t n_fixed, int mem);
void dyn_step(Elastodynamics* d, afem_solve_stats* st);
void dyn_set_dirichlet(Elastodynamics* d, const int32_t* dofs, const double* values, int64_t n, int mem);
void dyn_set_time_step(Elastodynamics* d, double dt);
void dyn_profile(Elastodynamics* d, bool on);
void dyn_destroy(Elastodynamics* d);

void vec_lincomb(Ctx& ctx, int64_t n, double a, const double* x, double b, const double* y, double c, const double* z,
                 double* out);
void newmark_update(Ctx& ctx, int64_t n, double dt, double beta, double gamma, const double* un, double* u, double* v,
                    double* a);
// x[ids[i]] = vals[i] (device arrays)
void vec_scatter(Ctx& ctx, int64_t n, const int32_t* ids, const double* vals, double* x);

void comm_unique_id(uint8_t* out);
Comm* comm_create(Ctx& ctx, const uint8_t* id, int nranks, int rank);
Comm* comm_create_host(int nranks, int rank, const afem_host_transport* t);
void comm_destroy(Comm* c);
int comm_nranks(Comm* c);
int comm_rank(Comm* c);
void halo_setup(Halo& h, Ctx& ctx, Comm* comm, int n_nbr, const int32_t* nbr, const int64_t* send_cnt,
                const int32_t* send_ids, const int64_t* recv_cnt, const int32_t* recv_ids);

}  // namespace afem

// Opaque C handles map 1:1 to the internal objects.
struct afem_ctx : afem::Ctx {};
struct afem_mesh : afem::Mesh {};
struct afem_bsr : afem::Bsr {};
struct afem_ls : afem::LinearSystem {};
struct afem_comm {
  afem::Comm* c = nullptr;
  afem::Ctx* ctx = nullptr;
};
struct afem_elastodynamics {
  afem::Elastodynamics* d = nullptr;
};
