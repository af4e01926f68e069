/*
 * arcanefem_amd_generic.hpp -- generic element-functor assembly on libafem's
 * structure (HIP C++, header-only; compile the caller with hipcc
 * --offload-arch=gfx950).
 *
 * The reference's BSRFormat<NB_DOF>::assembleBilinear(compute_element_matrix)
 * (femutils/BSRFormat.h:786-837, 937-1100, 1105-1111) takes the module's
 * element functor -- e.g. modules/poisson/FemModule.cc:269-271:
 *     [=] ARCCORE_HOST_DEVICE (CellLocalId c) { return _computeElementMatrixTetra4Gpu(c, cn_cv, in_node_coord); }
 * -- and scatters the returned (NV*NB_DOF)^2 FixedMatrix into the BSR values
 * cell by cell (owned rows only, column found by a linear search of the row,
 * doAtomic<Add>).  afem::generic::assemble_bilinear<NV, NB_DOF>(bsr, f) is
 * that entry for ANY device functor f(int32_t cell) whose result has
 * operator()(int, int), on CDNA4 terms (k_assemble_units below):
 *
 *   - one wavefront owns a UNIT of the structure's cell-unit plan
 *     (afem_bsr_functor_plan, libafem functor_plan.hip): a column of 8 x 8
 *     lattice nodes over a segment of z layers (meshes on a lattice), else a
 *     64/NB_DOF^2-row piece of a processing-order slice;
 *   - the k x k blocks of the unit's rows live in LDS (two node layers at a
 *     time); each lane evaluates f for one cell of the current stage,
 *     coalesced 16-B entry loads carry the cell id, the lane that owns each
 *     vertex's row and the vertex's slot in every row: the element's rows go
 *     into LDS with ds_add_f64 (wavefront-local atomics, one wave per unit, in
 *     program order: the summation order of every value is fixed, so the
 *     result is bitwise reproducible -- the reference's global atomics are
 *     not), no column search, no global atomics;
 *   - when a layer is complete its rows are written to HBM once: runs of 8
 *     consecutive rows as contiguous stores through a flat LDS image,
 *     otherwise per row.
 *
 * f is evaluated once per (unit, cell): 1.34x per cell on an 8 x 8 x 10
 * lattice column (the cells shared with the neighbour columns and segments),
 * against 1x for the atomic scatter and 4x for the reference's atomic-free
 * gather.  Mode::Accumulate adds to the current values like the reference
 * (afem_bsr_reset_values zeroes them); Mode::Overwrite writes the element sums
 * (the values need no zeroing: assembly after resetMatrixValues in one pass).
 *
 * assemble_bilinear_atomic is the reference's algorithm (one lane per cell,
 * binary search of the sorted row, f64 atomics into HBM; summation order not
 * fixed): the fallback when a plan's LDS tile does not fit, kept for
 * comparison.  The fixed-physics entries (afem_bsr_assemble_poisson_p1 /
 * _elasticity_p1) stay the fastest instances: their element arithmetic is
 * compiled into the row-strip kernels.
 *
 * The functor sees the cell id; for geometry it captures the device arrays of
 * afem_bsr_assembly_view (cell_node, coords: the mesh's own numbering) or its
 * own (an Arcane shim captures Arcane's views: cell ids are the caller's).
 */
#ifndef ARCANEFEM_AMD_GENERIC_HPP
#define ARCANEFEM_AMD_GENERIC_HPP

#include <hip/hip_runtime.h>

#include "arcanefem_amd.h"

namespace afem {
namespace generic {

/* FixedMatrix<N, M> of femutils/FemUtils.h:53-186 (row-major, host+device): a
 * result type a functor may return; any type with operator()(int, int) works. */
template <int N, int M>
struct FixedMatrix {
  double v[N * M];
  __host__ __device__ double& operator()(int i, int j) { return v[i * M + j]; }
  __host__ __device__ double operator()(int i, int j) const { return v[i * M + j]; }
};

/* The structure a generic kernel scatters into (device pointers). */
struct CellAccess {
  const int32_t* cell_node;
  const double* coords;
  __device__ int32_t node(int32_t cell, int i, int nv) const { return cell_node[(int64_t)cell * nv + i]; }
  __device__ double x(int32_t node, int c) const { return coords[3 * (int64_t)node + c]; }
};

enum class Mode : int {
  Accumulate = 0, /* values += element sums (BSRFormat::assembleBilinear) */
  Overwrite = 1   /* values  = element sums (resetMatrixValues + assembleBilinear in one pass) */
};

/* ------------------------------------------------------------ unit kernel */

/* One wavefront per block: its LDS operations execute in issue order, so the
 * phases of a unit (adds -> flush reads -> image -> stores -> zero fill) need
 * only the compiler to keep their order, not the lgkmcnt(0) drain of
 * __syncthreads.  Measured equal here (r04at: 1.89-1.90 ms with the module's
 * element, the kernel waits on its gathers, not on LDS), so the default stays
 * __syncthreads; define AFEM_GENERIC_WAVESYNC 1 for the wave-scope order. */
#ifndef AFEM_GENERIC_WAVESYNC
#define AFEM_GENERIC_WAVESYNC 0
#endif
__device__ __forceinline__ void unit_lds_order()
{
#if AFEM_GENERIC_WAVESYNC
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
#else
  __syncthreads();
#endif
}

/* A value store of the flush: non-temporal when it overwrites (the launch
 * never re-reads the values; they would evict the coordinates and entries the
 * next units read from L2).  AFEM_GENERIC_NT 0: plain stores. */
#ifndef AFEM_GENERIC_NT
#define AFEM_GENERIC_NT 1
#endif
/* AFEM_GENERIC_DIAG (diagnostic builds, values wrong): bit 1 no LDS adds (the
 * element entries summed into a register instead), bit 2 no value stores in
 * the flush -- where the unit kernel's time goes (tools/generic_ab.py with
 * AFEM_GENERIC_LIB pointing at such a build). */
#ifndef AFEM_GENERIC_DIAG
#define AFEM_GENERIC_DIAG 0
#endif
__device__ __forceinline__ void flush_store(double* d, double val, int overwrite)
{
#if AFEM_GENERIC_DIAG & 2
  if (val != 12345.678) return;  // (never taken: keeps the LDS reads)
#endif
#if AFEM_GENERIC_NT
  if (overwrite) {
    __builtin_nontemporal_store(val, d);
    return;
  }
#endif
  *d = overwrite ? val : *d + val;
}

/* Writes layer L of unit U (its LDS buffer) to the values and zeroes the buffer. */
template <int K, bool WIDE>
__device__ __forceinline__ void flush_layer(const afem_functor_plan& p, const afem_functor_unit& U, int L,
                                            double* __restrict__ acc, int bufsz, int sr, int swz, int lane, int overwrite)
{
  constexpr int KK = K * K;
  const int RL = p.rows_per_layer;
  double* buf = acc + (p.nbuf == 2 ? (L & 1) * bufsz : 0);
  const int32_t row = lane < RL ? p.layer_rows[(U.first_stage + L) * RL + lane] : -1;
  int64_t rb = 0;
  int len = 0;
  if (row >= 0) {
    rb = p.rows[row];
    len = (int)(p.rows[row + 1] - rb);
  }
  if (K == 1 && !WIDE && (U.flags & 1)) {
    // runs of 8 consecutive rows per 8 lanes: one contiguous value range each
    double v[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) v[s] = s < len ? buf[s * sr + (lane ^ (s & swz))] : 0.0;
    const long long rb0 = __shfl((long long)rb, lane & ~7);
    long long end = row >= 0 ? (long long)(rb + len) : rb0;
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
      const long long t = __shfl_xor(end, o);
      end = t > end ? t : end;
    }
    const int glen = (int)(end - rb0);
    int my_off = 0;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const int gl = __shfl(glen, 8 * g);
      if (g < (lane >> 3)) my_off += gl;
    }
    unit_lds_order();
    if (row >= 0) {
      const int o = my_off + (int)(rb - rb0);
#pragma unroll
      for (int s = 0; s < 16; ++s)
        if (s < len) buf[o + s] = v[s];
    }
    unit_lds_order();
    int ib = 0;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const long long dst = __shfl(rb0, 8 * g);
      const int gl = __shfl(glen, 8 * g);
      for (int q = lane; q < gl; q += 64) {
        flush_store(p.values + dst + q, buf[ib + q], overwrite);
      }
      ib += gl;
    }
    unit_lds_order();
  }
  else if (K == 1 && swz == 15) {
    // rows of arbitrary places (slice pieces, clusters): each row's values are one
    // contiguous range; 16 lanes store 16 consecutive values of one row (4 rows per
    // instruction) instead of every lane its own row (64 scattered 8-B stores).
    // The planes are XOR-swizzled by the slot (row' = row ^ (slot & 15)), so the 16
    // lanes reading one row across 16 planes hit 16 distinct banks.  Measured (r06q,
    // AFEM_GENERIC_DIAG=2, L-shape-3D refined 6x): the per-lane stores cost 0.45 ms
    // of 2.98 with the module's element, 0.88 of 2.90 with the lean one; this flush:
    // 3.10 -> 2.74 and 2.99 -> 2.38 ms (r06r/r06s; one stream of the layer's segments,
    // a lane per value found by a binary search over the offsets: 2.95 / 2.62 ms)
    const int sub = lane & 15;
#pragma unroll 4
    for (int g = 0; g < 16; ++g) {
      const int L = 4 * g + (lane >> 4);
      const long long rbL = __shfl((long long)rb, L);
      const int lenL = __shfl(len, L);
      for (int s = sub; s < lenL; s += 16) flush_store(p.values + rbL + s, buf[s * sr + (L ^ (s & 15))], overwrite);
    }
  }
  else if (row >= 0) {
    for (int s = 0; s < len; ++s)
#pragma unroll
      for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const int pl = s * KK + i * K + j;
          const double val = buf[pl * sr + (lane ^ (pl & swz))];
          const int64_t idx = p.ordered_per_block ? (rb + s) * KK + i * K + j
                                                  : rb * KK + (int64_t)i * K * len + K * s + j;
          flush_store(p.values + idx, val, overwrite);
        }
  }
  unit_lds_order();
  for (int i = lane; i < bufsz; i += 64) buf[i] = 0.0;
  unit_lds_order();
}

/* One wavefront per unit (blockDim 64); dynamic LDS: nbuf * width * K^2 * sr
 * doubles, layout [buffer][slot*K^2 + i*K + j][row], planes of sr =
 * rows_per_layer + pad rows (pad 1 puts the slots of one row on different
 * LDS banks -- the cells of one ds_add_f64 share rows, not slots -- but its
 * 16.6 KB per unit leave 9 waves per CU instead of 10: 3 % slower at C2, so
 * the default is 0); pad < 0 keeps the dense planes and XOR-swizzles the rows
 * of plane pl by pl mod 16 instead (row' = row ^ (pl & swz)).
 *
 * UN functor evaluations per lane are in flight at once (entries e, e + 64,
 * ..., e + 64 (UN-1) of the stage): the UN cells' connectivity and coordinate
 * gathers issue together before any element is scattered, so a wave waits for
 * one chain of dependent loads per UN cells (the kernel is load-latency bound:
 * 16 KB of LDS per unit leave 2-3 waves per SIMD).  The scatter order stays
 * the one-cell-at-a-time order (entry e's adds, then e + 64's, ...): the same
 * bits for every UN. */
#ifndef AFEM_GENERIC_WAVES
#define AFEM_GENERIC_WAVES 0
#endif
#if AFEM_GENERIC_WAVES > 0
#define AFEM_GENERIC_WAVES_ATTR __attribute__((amdgpu_waves_per_eu(AFEM_GENERIC_WAVES)))
#else
#define AFEM_GENERIC_WAVES_ATTR
#endif
template <int NV, int K, bool WIDE, bool PK, int SR, int UN, class F>
__global__ void __launch_bounds__(64) AFEM_GENERIC_WAVES_ATTR k_assemble_units(afem_functor_plan p, F f, int sr_arg, int swz_arg,
                                                                               int overwrite)
{
  // SR > 0: planes of SR rows, no swizzle, compiled in (the LDS address of an
  // add is one shift-add of its slot); 0: the arguments
  const int sr = SR ? SR : sr_arg;
  const int swz = SR ? 0 : swz_arg;
  extern __shared__ __align__(16) double acc[];
  constexpr int KK = K * K;
  const int lane = threadIdx.x;
  // XCD-aware: blocks go round-robin over the 8 XCDs; XCD x takes the x-th
  // contiguous eighth of the units (neighbouring columns share one L2)
  const int64_t n = p.n_units, bid = blockIdx.x;
  const int64_t q = n >> 3, rem = n & 7, x = bid & 7, j = bid >> 3;
  const int64_t u = x * q + (x < rem ? x : rem) + j;
  const afem_functor_unit U = p.units[u];
  const int bufsz = p.width * KK * sr;
  for (int i = lane; i < p.nbuf * bufsz; i += 64) acc[i] = 0.0;
  unit_lds_order();
  // the lane's entries of the next group are loaded one group ahead (the next
  // group of this stage, else the first group of the next stage), so their
  // latency hides behind the functors; tagged with the group's first entry (a
  // stage without entries breaks the chain: the next one loads in place)
  uint4 nxt[UN];
  uint2 nxt2[UN];
  int64_t nxt_base = -1;
#if AFEM_GENERIC_DIAG & 1
  double diag_sink = 0.0;
#endif
  for (int L = 0; L < U.n_stages; ++L) {
    const int64_t e0 = p.stage_ptr[U.first_stage + L], e1 = p.stage_ptr[U.first_stage + L + 1];
    const int64_t e2 = L + 1 < U.n_stages ? p.stage_ptr[U.first_stage + L + 2] : e1;
    for (int64_t eb = e0; eb < e1; eb += 64 * UN) {
      uint4 m[UN];
      uint2 m2[UN];
      const bool have = nxt_base == eb;
#pragma unroll
      for (int v = 0; v < UN; ++v) {
        const int64_t e = eb + 64 * v + lane;
        m[v] = uint4{};
        m2[v] = uint2{};
        if (e < e1) {
          if (have) {
            m[v] = nxt[v];
            if (WIDE || PK) m2[v] = nxt2[v];
          }
          else if (PK) {  // a chain break: entry and pattern in place
            m2[v] = reinterpret_cast<const uint2*>(p.entries)[e];
            m[v] = reinterpret_cast<const uint4*>(p.patterns)[m2[v].y];
          }
          else {
            m[v] = reinterpret_cast<const uint4*>(p.entries)[e];
            if (WIDE) m2[v] = reinterpret_cast<const uint2*>(p.entries2)[e];
          }
        }
      }
      const bool more = eb + 64 * UN < e1;
      const int64_t nb = more ? eb + 64 * UN : e1, lim = more ? e1 : e2;
      nxt_base = lim > nb ? nb : -1;
#pragma unroll
      for (int v = 0; v < UN; ++v) {
        const int64_t en = nb + 64 * v + lane;
        if (en < lim) {
          if (PK) {
            nxt2[v] = reinterpret_cast<const uint2*>(p.entries)[en];
          }
          else {
            nxt[v] = reinterpret_cast<const uint4*>(p.entries)[en];
            if (WIDE) nxt2[v] = reinterpret_cast<const uint2*>(p.entries2)[en];
          }
        }
      }
      if (eb + lane < e1) {  // else no entry for this lane (then none of its later ones either)
        uint32_t cell[UN], pos[UN], sl[UN][4];
#pragma unroll
        for (int v = 0; v < UN; ++v) {
          if (WIDE) {
            sl[v][0] = m[v].x;
            sl[v][1] = m[v].y;
            sl[v][2] = m[v].z;
            sl[v][3] = m[v].w;
            cell[v] = m2[v].x;
            pos[v] = m2[v].y;
          }
          else {
            cell[v] = PK ? m2[v].x : m[v].x;
            sl[v][0] = m[v].y & 0xffffu;
            sl[v][1] = m[v].y >> 16;
            sl[v][2] = m[v].z & 0xffffu;
            sl[v][3] = m[v].z >> 16;
            pos[v] = m[v].w;
          }
        }
        // a lane past the stage's end evaluates its first cell again (pure
        // functor) and scatters nothing for it: no branch between the functors
        decltype(f(0)) ke[UN];
#pragma unroll
        for (int v = 0; v < UN; ++v) ke[v] = f((int32_t)(eb + 64 * v + lane < e1 ? cell[v] : cell[0]));
#pragma unroll
        for (int v = 0; v < UN; ++v) {
          if (eb + 64 * v + lane >= e1) break;
#pragma unroll
          for (int a = 0; a < NV; ++a) {
            const uint32_t pa = (pos[v] >> (8 * a)) & 0xffu;
            if (!(pa & 0x80u)) continue;
            double* const bufp = acc + ((pa >> 6) & 1u) * bufsz;
            const int row = (int)(pa & 63u);
#pragma unroll
            for (int b = 0; b < NV; ++b) {
              const int s = WIDE ? (int)((sl[v][a] >> (8 * b)) & 0xffu) : (int)((sl[v][a] >> (4 * b)) & 0xfu);
#pragma unroll
              for (int i = 0; i < K; ++i)
#pragma unroll
                for (int jj = 0; jj < K; ++jj) {
                  const int pl = s * KK + i * K + jj;
#if AFEM_GENERIC_DIAG & 1
                  diag_sink += (double)ke[v](K * a + i, K * b + jj) + (double)(pl * sr + row);
#else
                  atomicAdd(bufp + pl * sr + (row ^ (pl & swz)), (double)ke[v](K * a + i, K * b + jj));
#endif
                }
            }
          }
        }
      }
      // packed: the next group's patterns (L2-resident table), issued after
      // this group's work so that its entries have arrived: the dependent load
      // hides behind the next group's functors like the entries do
      if (PK) {
#pragma unroll
        for (int v = 0; v < UN; ++v)
          if (nb + 64 * v + lane < lim) nxt[v] = reinterpret_cast<const uint4*>(p.patterns)[nxt2[v].y];
      }
    }
    unit_lds_order();
    if (L > 0) flush_layer<K, WIDE>(p, U, L - 1, acc, bufsz, sr, swz, lane, overwrite);
  }
  flush_layer<K, WIDE>(p, U, U.n_stages - 1, acc, bufsz, sr, swz, lane, overwrite);
#if AFEM_GENERIC_DIAG & 1
  if (diag_sink == 12345.678) p.values[0] = diag_sink;  // (never taken: keeps the functors)
#endif
}

/* Functor evaluations in flight per lane: 4 for element matrices up to 4 x 4
 * (register room: the unit's LDS, not its VGPRs, bounds the occupancy; C2
 * with the Poisson module's tet4 element, tools/generic_ab.py r04o: UN 1 /
 * 2 / 3 / 4 / 6 / 8 = 2.16 / 1.87 / 1.88 / 1.79 / 1.98 / 2.85 ms -- 6 and 8
 * cost waves: 224 and 256 VGPRs), 1 for the larger blocks (a 12 x 12 matrix
 * is 288 VGPRs). */
#ifndef AFEM_GENERIC_UNROLL
#define AFEM_GENERIC_UNROLL 4
#endif
#ifndef AFEM_GENERIC_PAD
#define AFEM_GENERIC_PAD 0
#endif
/* the coalesced flush of units without a lattice (flush_layer; 0: the per-lane row stores) */
#ifndef AFEM_GENERIC_TRFLUSH
#define AFEM_GENERIC_TRFLUSH 1
#endif
constexpr int default_unroll(int nk) { return nk * nk <= 16 ? AFEM_GENERIC_UNROLL : 1; }

/* ------------------------------------------------------------ atomic kernel */

template <int NV, int K, class F>
__global__ void __launch_bounds__(256) k_assemble_cells(afem_assembly_view v, F f)
{
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= v.n_cells) return;
  const auto ke = f((int32_t)c);
  int32_t nodes[NV];
#pragma unroll
  for (int a = 0; a < NV; ++a) nodes[a] = v.cell_node[c * NV + a];
#pragma unroll
  for (int a = 0; a < NV; ++a) {
    const int32_t r = nodes[a];
    if (r < 0 || r >= v.n_rows) continue;  // isOwn(row): owned rows only
    const int64_t rb = v.rows[r], re = v.rows[r + 1];
#pragma unroll
    for (int b = 0; b < NV; ++b) {
      const int32_t col = nodes[b];
      int64_t lo = rb, hi = re;  // sorted row: lower bound of col
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (v.columns[mid] < col)
          lo = mid + 1;
        else
          hi = mid;
      }
      if (lo >= re || v.columns[lo] != col) {  // not in the structure (BSRMatrix::findValueIndex throws)
        atomicOr(v.error_flag, 1);
        continue;
      }
#pragma unroll
      for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const int64_t idx = v.ordered_per_block ? lo * (K * K) + i * K + j
                                                  : rb * (K * K) + (int64_t)i * K * (re - rb) + K * (lo - rb) + j;
          atomicAdd(v.values + idx, (double)ke(K * a + i, K * b + j));
        }
    }
  }
}

/* The reference's assembleBilinearAtomic (one lane per cell, f64 atomics into
 * HBM).  Checks the error flag (one synchronisation) unless check == false. */
template <int NV, int K, class F>
int assemble_bilinear_atomic(afem_bsr* bsr, F f, Mode mode = Mode::Accumulate, bool check = true)
{
  afem_assembly_view v;
  int rc = afem_bsr_assembly_view(bsr, &v);
  if (rc != AFEM_OK) return rc;
  if (v.nb_node_per_cell != NV || v.block_size != K) return AFEM_ERR_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(v.stream);
  if (mode == Mode::Overwrite && (rc = afem_bsr_reset_values(bsr)) != AFEM_OK) return rc;
  if (hipMemsetAsync(v.error_flag, 0, sizeof(int32_t), st) != hipSuccess) return AFEM_ERR_HIP;
  if (v.n_cells > 0) {
    const unsigned blocks = (unsigned)((v.n_cells + 255) / 256);
    hipLaunchKernelGGL((k_assemble_cells<NV, K, F>), dim3(blocks), dim3(256), 0, st, v, f);
    if (hipGetLastError() != hipSuccess) return AFEM_ERR_HIP;
  }
  if (!check) return AFEM_OK;
  int32_t flag = 0;
  if (hipMemcpyAsync(&flag, v.error_flag, sizeof(flag), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return AFEM_ERR_HIP;
  return flag ? AFEM_ERR_NOT_FOUND : AFEM_OK;
}

/* BSRFormat<K>::assembleBilinear(f) for cells of NV nodes: returns AFEM_OK or
 * an AFEM_ERR_* code (afem_last_error() tells why for library errors).
 * Enqueued on the structure's context stream, no synchronisation; the first
 * call builds the structure's cell-unit plan (afem_bsr_functor_plan, one
 * time).  Couplings outside the sparsity cannot occur: the plan is built from
 * the same cells as the structure. */
template <int NV, int K, int UN, class F>
int assemble_bilinear_unrolled(afem_bsr* bsr, F f, Mode mode = Mode::Accumulate, int pad = AFEM_GENERIC_PAD)
{
  afem_functor_plan p;
  int rc = afem_bsr_functor_plan(bsr, &p);
  if (rc != AFEM_OK) return rc;
  if (p.nb_node_per_cell != NV || p.block_size != K) return AFEM_ERR_ARG;
  // pad < 0: no padding, the rows of plane pl XOR-swizzled by pl mod 16 instead
  // (power-of-two planes of at least 16 rows)
  const int RL = p.rows_per_layer;
  // units of arbitrary rows (no lattice; K = 1, 64 rows): XOR-swizzled planes, for
  // the coalesced flush (flush_layer)
  const bool tr = !p.lattice && K == 1 && RL == 64 && AFEM_GENERIC_TRFLUSH;
  const int swz = tr || (pad < 0 && RL >= 16 && (RL & (RL - 1)) == 0) ? 15 : 0;
  if (pad < 0 || tr) pad = 0;
  int sr = p.rows_per_layer + pad;
  size_t lds = (size_t)p.nbuf * p.width * K * K * sr * sizeof(double);
  if (lds > 64 * 1024 && pad) {  // no room for the padding: dense planes
    sr = p.rows_per_layer;
    lds = (size_t)p.nbuf * p.width * K * K * sr * sizeof(double);
  }
  if (lds > 64 * 1024) return assemble_bilinear_atomic<NV, K>(bsr, f, mode, true);
  if (p.n_units == 0) return AFEM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(p.stream);
  const int ow = mode == Mode::Overwrite ? 1 : 0;
  const dim3 grid((unsigned)p.n_units);
  const bool dense64 = sr == 64 && swz == 0;  // lattice columns of 8 x 8 rows (k = 1)
  if (p.wide)
    hipLaunchKernelGGL((k_assemble_units<NV, K, true, false, 0, UN, F>), grid, dim3(64), lds, st, p, f, sr, swz, ow);
  else if (p.packed && dense64)
    hipLaunchKernelGGL((k_assemble_units<NV, K, false, true, 64, UN, F>), grid, dim3(64), lds, st, p, f, sr, swz, ow);
  else if (p.packed)
    hipLaunchKernelGGL((k_assemble_units<NV, K, false, true, 0, UN, F>), grid, dim3(64), lds, st, p, f, sr, swz, ow);
  else if (dense64)
    hipLaunchKernelGGL((k_assemble_units<NV, K, false, false, 64, UN, F>), grid, dim3(64), lds, st, p, f, sr, swz, ow);
  else
    hipLaunchKernelGGL((k_assemble_units<NV, K, false, false, 0, UN, F>), grid, dim3(64), lds, st, p, f, sr, swz, ow);
  return hipGetLastError() == hipSuccess ? AFEM_OK : AFEM_ERR_HIP;
}

template <int NV, int K, class F>
int assemble_bilinear(afem_bsr* bsr, F f, Mode mode = Mode::Accumulate)
{
  return assemble_bilinear_unrolled<NV, K, default_unroll(NV * K)>(bsr, f, mode);
}

}  // namespace generic
}  // namespace afem

#endif /* ARCANEFEM_AMD_GENERIC_HPP */
