// P1 global-matrix assembly (the hot path; replaces the cell-wise atomic
// scatter of BSRFormat::assembleBilinearOrderedPerBlock/PerRow,
// femutils/BSRFormat.h:786-898, and the RHS source term of
// femutils/ArcaneFemFunctionsGpu.h:401-429).
//
// Design: a wavefront owns a slice of 64 rows (a 4x4x4
// node brick on structured meshes) and stages in LDS the coordinates of the
// nodes those rows couple to plus the rows' local column indices.  Each lane
// owns one row and walks the row's incident cells through the row-local
// incidence table (sliced ELL, one coalesced 1-KiB wave load per 4 steps).
// An incidence gives the row-slots of the cell's other nodes; the lane reads
// their coordinates from LDS, recomputes the element row K_e[row node, :] and
// accumulates it into the row's LDS accumulators.  The diagonal and the RHS
// are accumulated in registers; the finished rows are written once.
// Consequences:
//   * every value is written exactly once, no zero-fill pass, no float
//     atomics (global f64 atomics run at ~1.3 TB/s at best and ~0.08 TB/s
//     when 64 lanes hit 64 rows — the reference's access pattern);
//   * the summation order of every entry is fixed by the structure, so the
//     assembled matrix is bitwise reproducible run to run;
//   * HBM traffic ~= the algorithmic minimum: incidence table (4 B per
//     (cell,node), the same bytes as the connectivity), row offsets, columns,
//     values, RHS, coordinates once.
#include <cstring>
#include "afem_internal.hpp"

#include <cstdlib>
#include <type_traits>



namespace afem {
namespace {

constexpr uint32_t kPad = 0xFFFFFFFFu;

__device__ __forceinline__ int64_t xcd_swizzle(int64_t b, int64_t nb)
{
  // Blocks are dealt round-robin over the 8 XCDs (b and b+8 share one);
  // remap so each XCD walks a contiguous range of row blocks (L2 reuse of
  // the neighbouring rows' coordinates).  A bijection for any nb.
  const int64_t q = nb >> 3, rem = nb & 7;
  const int64_t x = b & 7, i = b >> 3;
  return x * q + (x < rem ? x : rem) + i;
}

struct V3 {
  double x, y, z;
};

__device__ __forceinline__ V3 ld3(const double* __restrict__ c, int64_t n)
{
  return V3{ c[3 * n + 0], c[3 * n + 1], c[3 * n + 2] };
}
// 1/a for the strip kernel: hardware estimate + ONE Newton step (relative
// error <= eps_rcp^2, below 2^-46 even for a 2^-23 estimate: far inside the
// 1e-12 parity bar; 3 VALU ops instead of 5)
__device__ __forceinline__ double recip1(double a)
{
  const double r = __builtin_amdgcn_rcp(a);
  return fma(r, fma(-a, r, 1.0), r);
}

__device__ __forceinline__ V3 sub(V3 a, V3 b) { return V3{ a.x - b.x, a.y - b.y, a.z - b.z }; }
// cross / dot with explicit fma: the same rounding in every kernel instance
// whatever the compiler's contraction choices (the strip instances agree bit
// for bit, tests/test_gpu_parity.py)
__device__ __forceinline__ V3 cross(V3 a, V3 b)
{
  return V3{ fma(a.y, b.z, -(a.z * b.y)), fma(a.z, b.x, -(a.x * b.z)), fma(a.x, b.y, -(a.y * b.x)) };
}
__device__ __forceinline__ double dot(V3 a, V3 b) { return fma(a.z, b.z, fma(a.y, b.y, a.x * b.x)); }

// 1/a to full double precision: hardware reciprocal estimate + two Newton
// steps (5 VALU ops instead of the ~10 of an IEEE division; within 1 ulp).
__device__ __forceinline__ double recip(double a)
{
  double r = __builtin_amdgcn_rcp(a);
  double e = fma(-a, r, 1.0);
  r = fma(r, e, r);
  e = fma(-a, r, 1.0);
  return fma(r, e, r);
}

// Element row of the P1 Laplacian for the row node x0 of a tetrahedron
// (x0,x1,x2,x3):  K_0b = V grad N_0 . grad N_b = (c_0 . c_b) / (6 |det|) with
// c_1 = e2 x e3, c_2 = e3 x e1, c_3 = e1 x e2, c_0 = -(c_1 + c_2 + c_3),
// e_k = x_k - x0 and det = e1 . c_1 = 6 V (signed).  Same quantity as
// modules/poisson/FemModule.h:177-186 with the gradients of
// femutils/ArcaneFemFunctionsGpu.h:280-392 (node order does not matter:
// the products are invariant under permutations and orientation).
// `s6` = coef/6, the returned |det| = 6V.
__device__ __forceinline__ double tet_row(V3 x0, V3 x1, V3 x2, V3 x3, double s6, double& k0, double& k1, double& k2,
                                          double& k3)
{
  const V3 e1 = sub(x1, x0), e2 = sub(x2, x0), e3 = sub(x3, x0);
  const V3 c1 = cross(e2, e3), c2 = cross(e3, e1), c3 = cross(e1, e2);
  const V3 c0 = V3{ -(c1.x + c2.x + c3.x), -(c1.y + c2.y + c3.y), -(c1.z + c2.z + c3.z) };  // sum of grads = 0
  const double det = fabs(dot(e1, c1));
  const double s = s6 * recip(det);
  k0 = dot(c0, c0) * s;
  k1 = dot(c0, c1) * s;
  k2 = dot(c0, c2) * s;
  k3 = dot(c0, c3) * s;
  return det;
}

// Triangle (x0,x1,x2) in the xy plane: grad N_a = c_a / A2 with
// c_1 = (e2.y, -e2.x), c_2 = (-e1.y, e1.x), c_0 = -(c_1 + c_2),
// K_0b = |A2|/2 * c_0.c_b / A2^2 = c_0.c_b / (2|A2|)
// (modules/poisson/FemModule.h:139-147, femutils/ArcaneFemFunctionsGpu.h:218-252).
// `s2` = coef/2, returns |A2| = 2 * area.
__device__ __forceinline__ double tri_row(V3 x0, V3 x1, V3 x2, double s2, double& k0, double& k1, double& k2)
{
  const double e1x = x1.x - x0.x, e1y = x1.y - x0.y, e2x = x2.x - x0.x, e2y = x2.y - x0.y;
  const double c1x = e2y, c1y = -e2x, c2x = -e1y, c2y = e1x;
  const double c0x = -(c1x + c2x), c0y = -(c1y + c2y);
  const double A2 = fabs(e1x * e2y - e2x * e1y);
  const double s = s2 * recip(A2);
  k0 = (c0x * c0x + c0y * c0y) * s;
  k1 = (c0x * c1x + c0y * c1y) * s;
  k2 = (c0x * c2x + c0y * c2y) * s;
  return A2;
}

// ---------------------------------------------------------------- slice tiles
// One wavefront per slice of 64 rows (Structure::perm).  LDS image of a
// slice, per wave:
//   acc [NACC*w_cap][64]  f64 accumulators, (slot, lane) at (slot*NACC + c)*64 + lane:
//                         a lane's ds_add_f64 hits its own bank pair, no conflicts;
//   cx, cy, (cz) [ucap]   coordinates of the slice's nodes (Structure::snode), SoA;
//   li [w_cap][64]        u16 index of the row's column `slot` in that list;
//   offs [2][64]          row offsets inside each run and row lengths (write-back).
// The coordinates of a cell's other nodes then come from LDS (3 ds_read_b64
// per node instead of 2 vector-memory gathers through the texture path,
// which bound the previous, row-contiguous version at ~85-92 % TA busy).
// UCAP > 0 fixes the coordinate array stride at compile time so that y and
// z are immediate offsets of the x address; the odd strides (257, 513, ...)
// keep the compiler from fusing the three reads into the half-rate
// ds_read2(st64)_b64 forms.  UCAP = 0: runtime stride.
__host__ __device__ constexpr int64_t tile_acc_bytes(int nacc, int64_t w_cap) { return 8 * 64 * (int64_t)nacc * w_cap; }
__host__ __device__ constexpr int64_t tile_coord_bytes(int dimc, int64_t u_cap)
{
  return (8 * (int64_t)dimc * u_cap + 15) & ~int64_t(15);
}
__host__ __device__ constexpr int64_t tile_bytes(int dimc, int nacc, int64_t u_cap, int64_t w_cap)
{
  return tile_acc_bytes(nacc, w_cap) + tile_coord_bytes(dimc, u_cap) + 2 * 64 * w_cap + 4 * 128;
}
constexpr int kUcapBuckets[4] = { 257, 513, 1025, 2049 };

template <int DIMC, int NACC, int UCAP>
struct Tile {
  double* acc;
  double* cx;
  uint16_t* li;
  int32_t* offs;
  int ucap;

  __device__ Tile(unsigned char* smem, int u_cap, int w_cap)
  {
    ucap = UCAP > 0 ? UCAP : u_cap;
    acc = reinterpret_cast<double*>(smem);
    cx = reinterpret_cast<double*>(smem + tile_acc_bytes(NACC, w_cap));
    li = reinterpret_cast<uint16_t*>(smem + tile_acc_bytes(NACC, w_cap) + tile_coord_bytes(DIMC, ucap));
    offs = reinterpret_cast<int32_t*>(reinterpret_cast<unsigned char*>(li) + 2 * 64 * w_cap);
  }
  __device__ __forceinline__ int stride() const { return UCAP > 0 ? UCAP : ucap; }

  // Coordinates of the nu slice nodes, the slice's index table (16-B copies
  // of W*128 bytes) and zeroed accumulators.  The index-table loads and the
  // node ids are issued first, then all coordinates (four nodes per lane per
  // round, one round for nu <= 256), then the LDS writes.  Lanes past an end
  // redo the last element (same value to the same address), so every load
  // and store is unconditional and none gets sunk behind an early wait.
  __device__ void stage(int lane, int nu, const int32_t* __restrict__ nodes, const double* __restrict__ coords, int W,
                        const uint16_t* __restrict__ lsrc)
  {
    const int st = stride();
    const uint4* src = reinterpret_cast<const uint4*>(lsrc);
    uint4* dst = reinterpret_cast<uint4*>(li);
    const int nq = 8 * W;
    const int q0 = min(lane, nq - 1), q1 = min(lane + 64, nq - 1);
    const uint4 l0 = src[q0], l1 = src[q1];
    for (int u = lane; u < nu; u += 256) {
      int idx[4];
      int64_t n[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        idx[k] = min(u + 64 * k, nu - 1);
        n[k] = nodes[idx[k]];
      }
      double x[4], y[4], z[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        x[k] = coords[3 * n[k]];
        y[k] = coords[3 * n[k] + 1];
        z[k] = DIMC == 3 ? coords[3 * n[k] + 2] : 0.0;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        cx[idx[k]] = x[k];
        cx[st + idx[k]] = y[k];
        if (DIMC == 3) cx[2 * st + idx[k]] = z[k];
      }
    }
    dst[q0] = l0;
    dst[q1] = l1;
    for (int q = lane + 128; q < nq; q += 64) dst[q] = src[q];
    double2* a2 = reinterpret_cast<double2*>(acc);
    for (int q = lane; q < 32 * NACC * W; q += 64) a2[q] = make_double2(0.0, 0.0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }

  __device__ __forceinline__ V3 node(int lane, uint32_t slot) const
  {
    const int u = li[slot * 64 + lane];
    const double* p = cx + u;
    return V3{ p[0], p[stride()], DIMC == 3 ? p[2 * stride()] : 0.0 };
  }
  __device__ __forceinline__ double* at(int lane, uint32_t slot, int c) const { return acc + (slot * NACC + c) * 64 + lane; }
};

__device__ __forceinline__ void wave_sync_lds()
{
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Coalesced write-back of a slice.  Lanes [j, j+run) hold consecutive rows
// (idle lanes only at the end of a run), so the run's value segments form
// one contiguous range [base_j, base_j + L_j): the wave writes it with
// consecutive lanes on consecutive addresses, each position's value taken
// from its row's accumulator column (owner found by a binary search over
// the run's row offsets).  NACC values per (row, slot): per block
// (slot*NACC + c) or, NACC = 4, per scalar row (i*2*len + 2*slot + j).
template <int NACC, class TILE>
__device__ __forceinline__ void write_back(const TILE& tile, int lane, int run, bool active, int64_t rb, int len,
                                           bool per_block, double* __restrict__ vals)
{
  const int j0 = lane & ~(run - 1);
  const int64_t base = __shfl(rb, j0);
  const int off = active ? (int)(rb - base) : 0x7fffffff;
  int end = active ? off + len : 0;
  for (int o = 1; o < run; o <<= 1) end = max(end, __shfl_xor(end, o));
  tile.offs[lane] = off;
  tile.offs[64 + lane] = len;
  wave_sync_lds();
  for (int j = 0; j < 64; j += run) {
    const int64_t bj = __shfl(base, j);
    const int lj = __shfl(end, j);
    for (int p = lane; p < NACC * lj; p += 64) {
      const int pr = p / NACC;  // scalar position of the block
      int q = 0;
      for (int step = run >> 1; step > 0; step >>= 1)
        if (tile.offs[j + q + step] <= pr) q += step;
      const int o = tile.offs[j + q];
      int slot, c;
      if (NACC == 1 || per_block) {
        slot = pr - o;
        c = p - NACC * pr;
      }
      else {  // per scalar row: the row's 4*len values are [i][slot][jj]
        const int w = p - NACC * o, rl2 = 2 * tile.offs[64 + j + q];
        const int i = w >= rl2 ? 1 : 0;
        const int rem = w - i * rl2;
        slot = rem >> 1;
        c = 2 * i + (rem & 1);
      }
      vals[NACC * bj + p] = *tile.at(j + q, slot, c);
    }
  }
}

// ---------------------------------------------------------------- scalar P1
// Incidence entry k of lane `lane` of slice `sl` lives at
// inc[slice_ptr[sl] + (k/4)*256 + lane*4 + k%4]: one 16-B load per lane per 4
// incidences, coalesced over the wave (1 KiB per load instruction).  A row
// is owned by a single lane and a wave's LDS operations execute in program
// order, so the summation order of every entry is fixed by the structure:
// the assembled matrix is bitwise reproducible run to run.
//
// Persistent, software-pipelined waves: a wave walks a contiguous chunk of
// slices (adjacent bricks: their coordinate footprints overlap in L1/L2).
// While it computes slice i, the loads of slice i+1 are in flight into
// registers (SlicePre): level 1 at the top of slice i (row ids, node ids,
// local column table, first incidence words), level 2 after the first
// incidence group (row offsets, row coordinates, node coordinates: they need
// the level-1 values).  Slice i+1 is then staged into LDS from registers with
// no memory wait, so the only exposed latency per slice is LDS latency.
// The write-back of slice i is a flat copy of its value segment (one
// contiguous range per x-run of rows) through a (position -> slot, lane) map
// built in the then-free column-table region; its stores retire under the
// next slice's arithmetic.
//
// The group loop is uniform over the wave (padding entries are computed as
// degenerate cells whose scale is masked to 0).  The diagonal is not
// accumulated: rows of the P1 Laplacian sum to zero (sum of the shape
// function gradients), so K_ii = -sum_{j != i} K_ij, formed before write-back.
// native 4 x u32 vector: plain registers (HIP's uint4 is a union-based class
// that keeps a struct copy of it in scratch)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Registers of one slice while it is in flight.  MAXG = incidence groups of 4
// held per lane (the whole incidence table row of the slice).
template <int MAXG>
struct SlicePre {
  int32_t row;
  int32_t len;
  int64_t rb;
  V3 xi;
  int32_t nid[4];
  u32x4 l0, l1;
  u32x4 wd[MAXG];
  double x[4], y[4], z[4];
};

// Every vector-memory operation of the steady state has a compile-time count
// (unrolled group loop, all incidence words prefetched, fixed-count
// unconditional write-back stores, clamped duplicate addresses instead of
// predication): the waitcnt pass can then wait for a load without draining
// the younger write-back stores (vmcnt retires in issue order).
// MAXW = max row length (slots) the fixed write-back covers.
template <int NV, int UCAP, int MAXG, int MAXW>
__global__ __launch_bounds__(64, 2) void k_assemble_p1(int64_t n_slices, int64_t chunk, int u_cap, int w_cap,
                                                    int64_t pad_off, const int32_t* __restrict__ perm,
                                                    const int64_t* __restrict__ row_ptr,
                                                    const uint32_t* __restrict__ inc,
                                                    const int64_t* __restrict__ slice_ptr,
                                                    const int32_t* __restrict__ slice_k,
                                                    const int32_t* __restrict__ slice_w,
                                                    const int64_t* __restrict__ lidx_ptr,
                                                    const uint16_t* __restrict__ lidx,
                                                    const int64_t* __restrict__ snode_ptr,
                                                    const int32_t* __restrict__ snode,
                                                    const double* __restrict__ coords, double s_coef,
                                                    double f_meas, double* __restrict__ vals,
                                                    double* __restrict__ rhs, int rhs_add)
{
  constexpr int DIMC = NV == 4 ? 3 : 2;
  extern __shared__ __align__(16) unsigned char smem[];
  Tile<DIMC, 1, UCAP> tile(smem, u_cap, w_cap);
  const int lane = threadIdx.x;
  int64_t sl = xcd_swizzle(blockIdx.x, gridDim.x) * chunk;
  const int64_t s_end = min(sl + chunk, n_slices);
  if (sl >= s_end) return;

  // level 1: everything addressed by slice scalars only
  auto level1 = [&](int64_t s, SlicePre<MAXG>& p) {
    p.row = perm[s * 64 + lane];
    const int nq = 8 * slice_w[s];
    const u32x4* ls = reinterpret_cast<const u32x4*>(lidx + lidx_ptr[s]);
    p.l0 = ls[max(min(lane, nq - 1), 0)];
    p.l1 = ls[max(min(lane + 64, nq - 1), 0)];
    const int64_t u0 = snode_ptr[s];
    const int nu = (int)(snode_ptr[s + 1] - u0);
#pragma unroll
    for (int k = 0; k < 4; ++k) p.nid[k] = snode[u0 + max(min(lane + 64 * k, nu - 1), 0)];
    const int ng = slice_k[s] >> 2;
    const int gl = ng > 0 ? ng - 1 : 0;
    const u32x4* ip = reinterpret_cast<const u32x4*>(inc + (ng > 0 ? slice_ptr[s] : pad_off)) + lane;
#pragma unroll
    for (int g = 0; g < MAXG; ++g) p.wd[g] = ip[(int64_t)min(g, gl) * 64];
  };
  // level 2: addressed by level-1 values
  auto level2 = [&](SlicePre<MAXG>& p) {
    const bool act = p.row >= 0;
    const int32_t r = act ? p.row : 0;
    const int64_t b = row_ptr[r];
    const int64_t e = row_ptr[r + 1];
    p.rb = act ? b : 0;
    p.len = act ? (int)(e - b) : 0;
    p.xi = ld3(coords, r);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      p.x[k] = coords[3 * (int64_t)p.nid[k]];
      p.y[k] = coords[3 * (int64_t)p.nid[k] + 1];
      p.z[k] = DIMC == 3 ? coords[3 * (int64_t)p.nid[k] + 2] : 0.0;
    }
  };

  SlicePre<MAXG> cur, nxt;
  level1(sl, cur);
  level2(cur);
  for (; sl < s_end; ++sl) {
    // the last slice of the chunk prefetches itself again (L2 hits): keeps
    // every load and the register hand-over unconditional
    const int64_t sn = sl + 1 < s_end ? sl + 1 : sl;
    const int ngroups = slice_k[sl] >> 2;  // uniform over the wave
    const int W = slice_w[sl];
    const int64_t u0 = snode_ptr[sl];
    const int nu = (int)(snode_ptr[sl + 1] - u0);

    // ---- stage slice sl from registers (+ the rare overflow beyond 256 nodes / 16 slots)
    {
      const int st = tile.stride();
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int idx = max(min(lane + 64 * k, nu - 1), 0);
        tile.cx[idx] = cur.x[k];
        tile.cx[st + idx] = cur.y[k];
        if (DIMC == 3) tile.cx[2 * st + idx] = cur.z[k];
      }
      if (nu > 256) {
        for (int u = lane + 256; u < nu; u += 64) {
          const int64_t n = snode[u0 + u];
          tile.cx[u] = coords[3 * n];
          tile.cx[st + u] = coords[3 * n + 1];
          if (DIMC == 3) tile.cx[2 * st + u] = coords[3 * n + 2];
        }
      }
      const int nq = 8 * W;
      u32x4* dst = reinterpret_cast<u32x4*>(tile.li);
      dst[max(min(lane, nq - 1), 0)] = cur.l0;
      dst[max(min(lane + 64, nq - 1), 0)] = cur.l1;
      if (nq > 128) {
        const u32x4* ls = reinterpret_cast<const u32x4*>(lidx + lidx_ptr[sl]);
        for (int q = lane + 128; q < nq; q += 64) dst[q] = ls[q];
      }
      double2* a2 = reinterpret_cast<double2*>(tile.acc);
      for (int q = lane; q < 32 * W; q += 64) a2[q] = make_double2(0.0, 0.0);
    }
    wave_sync_lds();
    level1(sn, nxt);

    const int32_t row = cur.row;
    const bool active = row >= 0;
    const int64_t rb = cur.rb;
    const int len = cur.len;
    const V3 xi = cur.xi;
    const uint32_t dslot = (ngroups == 0 || cur.wd[0].x == kPad) ? 0xFFu : (cur.wd[0].x >> 24);
    double macc = 0.0;

    auto group = [&](const u32x4 w) {
      const uint32_t ev[4] = { w.x, w.y, w.z, w.w };
      V3 xa[4], xb[4], xc[4];
      uint32_t sa[4], sb[4], sc[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t e = ev[j] == kPad ? 0u : ev[j];
        sa[j] = e & 0xFFu;
        sb[j] = (e >> 8) & 0xFFu;
        sc[j] = (NV == 4) ? (e >> 16) & 0xFFu : 0u;
        xa[j] = tile.node(lane, sa[j]);
        xb[j] = tile.node(lane, sb[j]);
        if (NV == 4) xc[j] = tile.node(lane, sc[j]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool pad = ev[j] == kPad;  // padding: degenerate cell (det 0), scale forced to 0
        double k1, k2, k3 = 0.0, meas;
        if (NV == 4) {
          const V3 e1 = sub(xa[j], xi), e2 = sub(xb[j], xi), e3 = sub(xc[j], xi);
          const V3 c1 = cross(e2, e3), c2 = cross(e3, e1), c3 = cross(e1, e2);
          const V3 c0 = V3{ -(c1.x + c2.x + c3.x), -(c1.y + c2.y + c3.y), -(c1.z + c2.z + c3.z) };
          meas = fabs(dot(e1, c1));
          const double s = pad ? 0.0 : s_coef * recip(meas);
          k1 = dot(c0, c1) * s;
          k2 = dot(c0, c2) * s;
          k3 = dot(c0, c3) * s;
        }
        else {
          const double e1x = xa[j].x - xi.x, e1y = xa[j].y - xi.y, e2x = xb[j].x - xi.x, e2y = xb[j].y - xi.y;
          const double c1x = e2y, c1y = -e2x, c2x = -e1y, c2y = e1x;
          const double c0x = -(c1x + c2x), c0y = -(c1y + c2y);
          meas = fabs(e1x * e2y - e2x * e1y);
          const double s = pad ? 0.0 : s_coef * recip(meas);
          k1 = (c0x * c1x + c0y * c1y) * s;
          k2 = (c0x * c2x + c0y * c2y) * s;
        }
        macc += meas;
        atomicAdd(tile.at(lane, sa[j], 0), k1);
        atomicAdd(tile.at(lane, sb[j], 0), k2);
        if (NV == 4) atomicAdd(tile.at(lane, sc[j], 0), k3);
      }
    };
    // unrolled over the compile-time group count (uniform skips past the
    // slice's width); the next slice's level-2 loads go out after group 1,
    // when its level-1 loads (issued a whole slice earlier) have landed
#pragma unroll
    for (int g = 0; g < MAXG; ++g) {
      if (g < ngroups) group(cur.wd[g]);
      if (g == 1) level2(nxt);
    }
    if (MAXG < 2) level2(nxt);

    // ---- RHS (unconditional store: idle lanes repeat an active lane's store)
    {
      const unsigned long long am = __ballot(active);
      const int src = active ? lane : (int)__ffsll((long long)am) - 1;
      const double rv = __shfl(f_meas * macc, src);
      const int32_t rr = __shfl(row, src);
      if (rhs) st_out(&rhs[rr], rhs_add ? rhs[rr] + rv : rv);
    }
    wave_sync_lds();

    // ---- diagonal + write-back.  Each lane pulls its row out of the
    // [slot][lane] accumulators into registers (conflict-free: a lane always
    // hits its own bank pair), forms the diagonal, and stores the row back in
    // CSR order at its flat offset (rows of one x-run of lanes are
    // consecutive, so the flat image of a slice is a few contiguous value
    // ranges).  Then consecutive lanes copy consecutive flat positions to
    // HBM: conflict-free LDS reads, coalesced stores.  The flat image reuses
    // the accumulator region, the (position -> slot, lane) map the
    // column-table region.
    int fp = len;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(fp, o);
      if (lane >= o) fp += t;
    }
    const int total = __shfl(fp, 63);
    fp -= len;
    uint16_t* map = tile.li;
    int64_t* rbs = reinterpret_cast<int64_t*>(tile.offs);
    if (W <= MAXW) {
      double rv[MAXW];
#pragma unroll
      for (int t = 0; t < MAXW; ++t) rv[t] = *tile.at(lane, min(t, W - 1), 0);
      double sum = 0.0;
#pragma unroll
      for (int t = 0; t < MAXW; ++t)
        if (t < len && t != (int)dslot) sum += rv[t];
#pragma unroll
      for (int t = 0; t < MAXW; ++t)
        if (t == (int)dslot) rv[t] = -sum;
      wave_sync_lds();  // every lane's reads before the overlapping flat writes
#pragma unroll
      for (int t = 0; t < MAXW; ++t)
        if (t < len) {
          tile.acc[fp + t] = rv[t];
          map[fp + t] = (uint16_t)(t * 64 + lane);
        }
      rbs[lane] = rb;
      wave_sync_lds();
#pragma unroll
      for (int k = 0; k < MAXW; ++k) {
        const int P = min(64 * k + lane, total - 1);
        const double v = tile.acc[P];
        const int m = map[P];
        st_out(&vals[rbs[m & 63] + (m >> 6)], v);
      }
    }
    else {  // rows longer than MAXW (not on the host-selected variants)
      if (active && dslot != 0xFFu) {
        double sum = 0.0;
        for (int t = 0; t < len; ++t)
          if (t != (int)dslot) sum += *tile.at(lane, t, 0);
        *tile.at(lane, dslot, 0) = -sum;
      }
      for (int t = 0; t < len; ++t) map[fp + t] = (uint16_t)(t * 64 + lane);
      rbs[lane] = rb;
      wave_sync_lds();
      for (int p = lane; p < total; p += 64) {
        const int ix = map[p];
        st_out(&vals[rbs[ix & 63] + (ix >> 6)], tile.acc[ix]);
      }
    }
    wave_sync_lds();
    cur = nxt;
  }
}


// ---------------------------------------------------------------- scalar P1, row strips
// Same slice tiles and software pipeline as k_assemble_p1, but each lane walks
// its row's strip (sparsity.hip "row strips"): one stream byte per cell gives
// the ONE new node of the window (slot + shift/swap kind).  Per cell: one
// coordinate gather (3 LDS reads instead of 9), one index read (instead of 3),
// two new cofactors (the third is the previous cell's, up to sign), ~42 FP64
// ops instead of 55; the stream is 1 B per step instead of 4 B per cell.
//   window (P,Q,R) + node D:  shift -> (Q,R,D),  swap -> (P,R,D)
//   cofactors c_P = e_Q x e_R, c_Q = e_R x e_P, c_R = e_P x e_Q (e = x - x_row):
//   c_R' = shift ? c_P : -c_Q (old window), c_P' = e_R x e_D, c_Q' = e_D x e_P'
//   K_row,b = coef (c_row . c_b) / (6 |det|), c_row = -(c_P + c_Q + c_R), det = e_P . c_P
// Triangles: window (P,Q) + D: shift -> (Q,D), swap -> (P,D).
// common step bytes of a uniform slice (sparsity.hip k_strip_classify): one
// s_load_dwordx8 per slice
struct alignas(32) SlotRec {
  uint32_t w[8];
};

template <int MAXC>
struct StripPre {
  int32_t row;
  uint32_t dl;  // diagonal slot | row length << 8
  int64_t rb;
  u32x4 l0, l1;
  u32x4 ch[MAXC];
  u32x4 cu[MAXC];  // uniform scalar instance: local node index of every step (strip_u)
  u32x4 pq;        // canonical structures: the row's slot map (Structure::cperm, 16 bytes)
  double x[4], y[4], z[4];
};
// byte t of a 16-byte slot map
__device__ __forceinline__ uint32_t pbyte(const u32x4& q, int t)
{
  const uint32_t w = (t >> 2) == 0 ? q.x : ((t >> 2) == 1 ? q.y : ((t >> 2) == 2 ? q.z : q.w));
  return (w >> (8 * (t & 3))) & 0xFFu;
}

// LDS image of a strip slice: accumulators [slot][lane] (as Tile), the
// slice's node coordinates AoS (DIMC doubles per node: one address per
// gather, components at immediate offsets), the u16 column-index table
// [slot][lane], 512 B of write-back scratch.
// (the coordinate region doubles as the write-back map: at least 4 B per value)
__host__ __device__ constexpr int64_t strip_coord_bytes(int dimc, int64_t u_cap, int64_t w_cap)
{
  return ((8 * (int64_t)dimc * u_cap > 256 * w_cap ? 8 * (int64_t)dimc * u_cap : 256 * w_cap) + 15) & ~int64_t(15);
}
__host__ __device__ constexpr int64_t strip_tile_bytes(int dimc, int64_t u_cap, int64_t w_cap)
{
  return 8 * 64 * w_cap + strip_coord_bytes(dimc, u_cap, w_cap) + 2 * 64 * w_cap + 512;
}
// block-3 tile: accumulators [slot][3][lane], coordinates (doubling as the
// u16 write-back map: 3 values per slot), column indices, per-lane value bases
__host__ __device__ constexpr int64_t elast_coord_bytes(int64_t u_cap, int64_t w_cap)
{
  return ((24 * u_cap > 6 * 64 * w_cap ? 24 * u_cap : 6 * 64 * w_cap) + 15) & ~int64_t(15);
}
__host__ __device__ constexpr int64_t elast_tile_bytes(int64_t u_cap, int64_t w_cap)
{
  return 3 * 8 * 64 * w_cap + elast_coord_bytes(u_cap, w_cap) + 2 * 64 * w_cap + 512;
}

#ifdef AFEM_WAVE_TIMES
// diagnostic build only (make EXTRA=-DAFEM_WAVE_TIMES OUT=../libafem_wt.so
// OBJDIR=build_wt; tools/wave_times.py): start / end realtime stamps and the
// slice count of every workgroup of the uniform strip instance
__device__ unsigned long long afem_wave_t[3 * 16384];
extern "C" int afem_debug_wave_times(unsigned long long* out, int n)
{
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(afem_wave_t), sizeof(unsigned long long) * (size_t)(3 * n));
}
#define AFEM_WT(i, v)                                                               \
  if (UMODE == 1 && lane == 0 && blockIdx.x < 16384) afem_wave_t[3 * blockIdx.x + (i)] = (v)
#else
#define AFEM_WT(i, v) (void)0
#endif

// UNI = true: the slices of `recs` (the uniform list) whose 64 rows share one strip topology
// (same length, one strip, same shift/swap sequence `spat`: every interior
// brick of a structured mesh).  The shift/swap decision is then wave-uniform:
// a scalar branch instead of 13 per-lane selects per step, the two priming
// steps only load the window, and no step needs an emit mask (≈45 instead of
// ≈72 VALU ops per cell).  Same formulas in the same order as the general
// path, so both give the same bits.
// PERM: a canonical structure (Structure::canon): the slots are the lattice's
// canonical ones and the write-back stores slot t at rb + cperm[16 p + t].
template <int NV, int MAXC, int MAXW, int UMODE, bool PERM = false>
__global__ __launch_bounds__(64, UMODE == 1 ? 3 : 2) void k_assemble_strip(int64_t n_slices, const SliceRec* __restrict__ recs,
                                                          unsigned long long* __restrict__ tickets,
                                                          int u_cap, int w_cap,
                                                          const int32_t* __restrict__ perm,
                                                          const int64_t* __restrict__ pos_rb,
                                                          const uint32_t* __restrict__ pos_dl,
                                                          const uint8_t* __restrict__ strip,
                                                          const uint8_t* __restrict__ strip_u,
                                                          const uint16_t* __restrict__ lidx,
                                                          const int32_t* __restrict__ snode,
                                                          const double* __restrict__ coords, double s_coef,
                                                          double f_meas, double* __restrict__ vals,
                                                          double* __restrict__ rhs, int rhs_add,
                                                          const SlotRec* __restrict__ uslots,
                                                          const uint8_t* __restrict__ cperm)
{
  // 1: scalar shift/swap branches, 2: selects on the uniform bit; 3: general
  // (per-lane) steps, but each step's node from the lane's local-index stream
  // (strip_u, slices of <= 256 nodes) instead of the column-index table
  constexpr bool UNI = UMODE == 1 || UMODE == 2;
  static_assert(!(PERM && UMODE == 1), "the slot map needs the select instance's register budget");
  // uniform tet instances address coordinates by the local-index stream (no
  // column-index table in LDS, no dependent LDS read per step)
  constexpr bool ULOC = (UNI && NV == 4) || UMODE == 3;
  constexpr bool USLOT = UNI && NV == 4;  // the slot bytes from the slice's common scalar stream
  constexpr int DIMC = NV == 4 ? 3 : 2;
  extern __shared__ __align__(16) unsigned char smem[];
  double* acc = reinterpret_cast<double*>(smem);
  double* cxyz = reinterpret_cast<double*>(smem + 8 * 64 * (int64_t)w_cap);
  uint16_t* li = reinterpret_cast<uint16_t*>(smem + 8 * 64 * (int64_t)w_cap + strip_coord_bytes(DIMC, u_cap, w_cap));
  int64_t* rbs = reinterpret_cast<int64_t*>(reinterpret_cast<unsigned char*>(li) + 2 * 64 * (int64_t)w_cap);
  const int lane = threadIdx.x;
  // Dynamic slice claiming, one ticket counter per XCD (workgroups are dealt
  // to the 8 XCDs round-robin): XCD x walks the contiguous x-th eighth of the
  // list, so neighbouring bricks stay in one L2.
  // Dynamic slice claiming, one ticket counter per XCD (workgroups are dealt
  // to the 8 XCDs round-robin): XCD x walks the contiguous x-th eighth of the
  // list, so neighbouring bricks stay in one L2.  (Cross-XCD stealing at the
  // end of the eighths, tried with a blocking re-claim, broke the scalar
  // record loads and the register budget of the pipeline; the XCDs finish
  // within ~5-10% of each other, tools/wave_times.py.)
  // issue: the atomic's result stays in a VGPR; get: readfirstlane (the list
  // position is provably wave-uniform: scalar loads, scalar branches).  In
  // the loop a claim is read one whole slice after it was issued, behind that
  // slice's stores, so the wave never waits on the atomic (or the stores).
  const int xcd = (int)(blockIdx.x & 7);
  const int64_t r0 = n_slices * xcd / 8, r1 = n_slices * (xcd + 1) / 8;
  auto claim_issue = [&]() -> unsigned long long {
    unsigned long long t = 0;
    if (lane == 0) t = atomicAdd(tickets + 16 * xcd, 1ull);
    return t;
  };
  auto claim_get = [&](unsigned long long t) -> int64_t {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)t);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(t >> 32));
    return r0 + (int64_t)(((uint64_t)hi << 32) | lo);
  };
#ifdef AFEM_WAVE_TIMES
  unsigned long long n_done = 0;
#endif
  // Four-stage software pipeline over the claimed list positions p0..p3:
  // while slice p0 is processed out of LDS, the row data, strip, column
  // indices and node coordinates of p1 are in flight, the node ids of p2
  // (the addresses of its coordinate gather), and the 32-B record of p3 (the
  // addresses of everything else).  Every dependent load thus has a whole
  // slice of work to land; positions past the end re-fetch p0 (never used).
  AFEM_WT(0, __builtin_amdgcn_s_memrealtime());
  int64_t p0 = claim_get(claim_issue());
  if (p0 >= r1) return;
  int64_t p1 = claim_get(claim_issue());
  int64_t p2 = claim_get(claim_issue());
  int64_t p3 = claim_get(claim_issue());
  SliceRec R0 = recs[p0];
  SliceRec R1 = recs[p1 < r1 ? p1 : p0];
  SliceRec R2 = recs[p2 < r1 ? p2 : p0];
  // uniform tet instances: the slot stream is common to the slice's rows (32
  // bytes per list position, scalar loads riding with the records)
  SlotRec S0{}, S1{}, S2{};
  if constexpr (USLOT) {
    S0 = uslots[p0];
    S1 = uslots[p1 < r1 ? p1 : p0];
    S2 = uslots[p2 < r1 ? p2 : p0];
  }

  auto load_nid = [&](const SliceRec& R, int32_t(&nid)[4]) {
    const int nu = (int)(R.meta & 0xFFFFu);
#pragma unroll
    for (int k = 0; k < 4; ++k) nid[k] = snode[(int64_t)R.snode_off + max(min(lane + 64 * k, nu - 1), 0)];
  };
  auto load_rows = [&](const SliceRec& R, StripPre<MAXC>& p) {
    const int64_t q = (int64_t)R.sl * 64 + lane;
    p.row = perm[q];
    p.dl = pos_dl[q];
    p.rb = pos_rb[q];
    if constexpr (PERM) p.pq = reinterpret_cast<const u32x4*>(cperm)[q];
    const int nc = (int)((R.meta >> 24) + 15) >> 4;
    if constexpr (!USLOT) {  // uniform instances read the slots from the scalar stream
      const u32x4* sp = reinterpret_cast<const u32x4*>(strip + (int64_t)R.strip_off * 1024) + lane;
#pragma unroll
      for (int c = 0; c < MAXC; ++c) p.ch[c] = sp[(int64_t)max(min(c, nc - 1), 0) * 64];
    }
    if constexpr (ULOC) {  // the steps' local node indices instead of the column-index table
      const u32x4* su = reinterpret_cast<const u32x4*>(strip_u + (int64_t)R.strip_off * 1024) + lane;
#pragma unroll
      for (int c = 0; c < MAXC; ++c) p.cu[c] = su[(int64_t)max(min(c, nc - 1), 0) * 64];
    }
    else {
      const int nq = 8 * (int)((R.meta >> 16) & 0xFFu);
      const u32x4* ls = reinterpret_cast<const u32x4*>(lidx + R.lidx_off);
      p.l0 = ls[max(min(lane, nq - 1), 0)];
      p.l1 = ls[max(min(lane + 64, nq - 1), 0)];
    }
  };
  auto gather = [&](const int32_t(&nid)[4], StripPre<MAXC>& p) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      p.x[k] = coords[3 * (int64_t)nid[k]];
      p.y[k] = coords[3 * (int64_t)nid[k] + 1];
      p.z[k] = DIMC == 3 ? coords[3 * (int64_t)nid[k] + 2] : 0.0;
    }
  };

  StripPre<MAXC> cur, nxt;
  int32_t nid1[4], nid2[4];
  {
    int32_t nid0[4];
    load_nid(R0, nid0);
    load_rows(R0, cur);
    gather(nid0, cur);
    load_nid(R1, nid1);
  }
  // drain the prologue loads: the loop header then inherits only the
  // back-edge's pending ops (loads a slice old, the stores), so the staging
  // waits count past the stores instead of on them
  __builtin_amdgcn_s_waitcnt(0);
  for (;;) {
    const unsigned long long t4 = claim_issue();    // read at the end of this iteration
    const SliceRec R3 = recs[p3 < r1 ? p3 : p0];    // scalar load, used two iterations later
    SlotRec S3{};
    if constexpr (USLOT) S3 = uslots[p3 < r1 ? p3 : p0];
    const int nsteps = (int)(R0.meta >> 24);  // uniform over the wave
    const int W = (int)((R0.meta >> 16) & 0xFFu);
    const int64_t u0 = R0.snode_off;
    const int nu = (int)(R0.meta & 0xFFFFu);

    // ---- stage slice p0 from registers (+ the rare overflow beyond 256 nodes / 16 slots)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int idx = max(min(lane + 64 * k, nu - 1), 0);
      cxyz[DIMC * idx] = cur.x[k];
      cxyz[DIMC * idx + 1] = cur.y[k];
      if (DIMC == 3) cxyz[DIMC * idx + 2] = cur.z[k];
    }
    if (!ULOC && nu > 256) {  // uniform / UMODE 3 slices: <= 256 nodes, <= 16 slots
      for (int u = lane + 256; u < nu; u += 64) {
        const int64_t n = snode[u0 + u];
        cxyz[DIMC * u] = coords[3 * n];
        cxyz[DIMC * u + 1] = coords[3 * n + 1];
        if (DIMC == 3) cxyz[DIMC * u + 2] = coords[3 * n + 2];
      }
    }
    {
      const int nq = 8 * W;
      u32x4* dst = reinterpret_cast<u32x4*>(li);
      if constexpr (!ULOC) {
        dst[max(min(lane, nq - 1), 0)] = cur.l0;
        dst[max(min(lane + 64, nq - 1), 0)] = cur.l1;
      }
      if (!ULOC && nq > 128) {
        const u32x4* ls = reinterpret_cast<const u32x4*>(lidx + R0.lidx_off);
        for (int q = lane + 128; q < nq; q += 64) dst[q] = ls[q];
      }
      double2* a2 = reinterpret_cast<double2*>(acc);
      for (int q = lane; q < 32 * W; q += 64) a2[q] = make_double2(0.0, 0.0);
    }
    wave_sync_lds();
    load_rows(R1, nxt);
    gather(nid1, nxt);
    load_nid(R2, nid2);

    const int32_t row = cur.row;
    const bool active = row >= 0;
    const int64_t rb = cur.rb;
    const int len = (int)((cur.dl >> 8) & 0xFFu);
    const uint32_t dslot = cur.dl & 0xFFu;
    // the row's own coordinates: its diagonal column is one of the slice's nodes
    const V3 xi = [&] {
      const double* q = cxyz + DIMC * (ULOC ? (int)(cur.dl >> 16) : (int)li[dslot * 64 + lane]);
      return V3{ q[0], q[1], DIMC == 3 ? q[2] : 0.0 };
    }();
    double macc = 0.0;
    // window state (zero vectors: finite arithmetic on priming / padding
    // steps); cN = e_P x e_R = -c_Q is kept instead of c_Q (no negations)
    V3 eP{ 0.0, 0.0, 0.0 }, eQ{ 0.0, 0.0, 0.0 }, eR{ 0.0, 0.0, 0.0 };
    V3 cP{ 0.0, 0.0, 0.0 }, cN{ 0.0, 0.0, 0.0 };
    double* const acc_lane = acc + lane;
    double* aP = acc_lane + 64 * dslot;  // accumulator addresses of the window nodes
    double* aQ = aP;
    double* aR = aP;
    const uint16_t* lrow = li + lane;

    auto lidx_of = [&](uint32_t byte) { return (int)lrow[(byte & 63u) * 64]; };
    auto coord = [&](int u) {
      const double* q = cxyz + DIMC * u;
      return V3{ q[0], q[1], DIMC == 3 ? q[2] : 0.0 };
    };
    auto sel = [](bool c, V3 a, V3 b) { return V3{ c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z }; };
    // x if the step emits a cell, +0.0 otherwise: a bit mask, not a select
    // (the compiler turns a select of a reciprocal into a branch)
    auto keep = [](uint64_t m, double x) { return __longlong_as_double((long long)(m & (uint64_t)__double_as_longlong(x))); };
    auto step = [&](uint32_t byte, V3 xd) {
      const bool swap = (byte & 0xC0u) == 0x40u;
      const uint64_t em = (uint64_t)0 - (uint64_t)(byte < 0x80u);
      double* const aD = acc_lane + 64 * (byte & 63u);
      const V3 eD = sub(xd, xi);
      double kP, kQ, kR = 0.0, meas;
      if (NV == 4) {
        const V3 cRn = sel(swap, cN, cP);  // c_R of the new window (shift: old c_P, swap: -old c_Q)
        eP = sel(swap, eP, eQ);
        aP = swap ? aP : aQ;
        eQ = eR;
        aQ = aR;
        eR = eD;
        aR = aD;
        cP = cross(eQ, eR);
        cN = cross(eP, eR);
        // -c_row = c_P + c_Q + c_R = c_P - cN + cRn
        const V3 m = V3{ cP.x - cN.x + cRn.x, cP.y - cN.y + cRn.y, cP.z - cN.z + cRn.z };
        meas = fabs(dot(eP, cP));
        const double s = keep(em, -s_coef * recip1(meas));  // carries the sign of c_row = -m
        kP = dot(m, cP) * s;
        kQ = -dot(m, cN) * s;
        kR = dot(m, cRn) * s;
      }
      else {
        eP = sel(swap, eP, eQ);
        aP = swap ? aP : aQ;
        eQ = eD;
        aQ = aD;
        // triangle (row, P, Q): c_P = (eQ.y, -eQ.x), c_Q = (-eP.y, eP.x), c_row = -(c_P + c_Q)
        const double cpx = eQ.y, cpy = -eQ.x, cqx = -eP.y, cqy = eP.x;
        const double crx = -(cpx + cqx), cry = -(cpy + cqy);
        meas = fabs(eP.x * eQ.y - eQ.x * eP.y);
        const double s = keep(em, s_coef * recip1(meas));
        kP = (crx * cpx + cry * cpy) * s;
        kQ = (crx * cqx + cry * cqy) * s;
      }
      macc += keep(em, meas);
      atomicAdd(aP, kP);
      atomicAdd(aQ, kQ);
      if (NV == 4) atomicAdd(aR, kR);
    };

    // steps: byte j of the stream = byte j%16 of chunk j/16; uniform guard per
    // 4-step word, padding steps are no-ops.  Two-deep LDS pipeline: at step
    // j the column-index read of step j+2 and the coordinate reads of step
    // j+1 are issued before step j's arithmetic and accumulator adds (no
    // alias hazard: coordinates and indices are not written in the loop).
    auto byte_at = [&](int j) -> uint32_t {
      if constexpr (USLOT) {  // scalar: the slice's common slot stream
        return (S0.w[(j >> 2) & 7] >> (8 * (j & 3))) & 0xFFu;
      }
      else {
        const u32x4 w = cur.ch[j >> 4];
        const int q = (j >> 2) & 3;
        const uint32_t wq = q == 0 ? w.x : (q == 1 ? w.y : (q == 2 ? w.z : w.w));
        return (wq >> (8 * (j & 3))) & 0xFFu;
      }
    };
    auto uloc_at = [&](int j) -> int {  // local node index of step j (ULOC)
      const u32x4 w = cur.cu[j >> 4];
      const int q = (j >> 2) & 3;
      const uint32_t wq = q == 0 ? w.x : (q == 1 ? w.y : (q == 2 ? w.z : w.w));
      return (int)((wq >> (8 * (j & 3))) & 0xFFu);
    };
    constexpr int NSTEP = 16 * MAXC;
    if constexpr (UNI && NV == 4) {
      // uniform strip: steps 0,1 prime the window (no cell), every later step
      // emits; the shift/swap bit is a scalar (one branch per step, both arms
      // straight-line code; only the kept node's registers move on a shift)
      const uint64_t pat = R0.pat;
      auto ustep = [&](auto swap_c, uint32_t byte, V3 xd, bool swp) {
        constexpr int SWAP = decltype(swap_c)::value;  // 1 swap, 0 shift, -1 select on swp
        double* const aD = acc_lane + 64 * (byte & 63u);
        const V3 eD = sub(xd, xi);
        V3 cRn;
        if constexpr (SWAP == 1) {
          cRn = cN;
        }
        else if constexpr (SWAP == 0) {
          cRn = cP;
          eP = eQ;
          aP = aQ;
        }
        else {
          cRn = sel(swp, cN, cP);
          eP = sel(swp, eP, eQ);
          aP = swp ? aP : aQ;
        }
        eQ = eR;
        aQ = aR;
        eR = eD;
        aR = aD;
        cP = cross(eQ, eR);
        cN = cross(eP, eR);
        const V3 m = V3{ cP.x - cN.x + cRn.x, cP.y - cN.y + cRn.y, cP.z - cN.z + cRn.z };
        // a padding step (odd lengths: the guard is every 2 steps) has a zero edge: meas = 0, all
        // k but the diagonal's (aR) exactly 0 with the finite 1/tiny
        const double meas = fabs(dot(eP, cP));
        const double s = -s_coef * recip1(fmax(meas, 1e-300));
        const double kP = dot(m, cP) * s;
        const double kQ = -dot(m, cN) * s;
        const double kR = dot(m, cRn) * s;
        macc += meas;
        atomicAdd(aP, kP);
        atomicAdd(aQ, kQ);
        atomicAdd(aR, kR);
      };
      {
        const uint32_t b0 = byte_at(0), b1 = byte_at(1);
        eQ = sub(coord(uloc_at(0)), xi);
        eR = sub(coord(uloc_at(1)), xi);
        aQ = acc_lane + 64 * (b0 & 63u);
        aR = acc_lane + 64 * (b1 & 63u);
        cP = cross(eQ, eR);
      }
      V3 xc = coord(uloc_at(2));
#pragma unroll
      for (int j = 2; j < NSTEP; ++j) {
        if ((j & (UMODE == 1 ? 1 : 3)) == 0 && j >= nsteps) break;
        const V3 xn = j + 1 < NSTEP ? coord(uloc_at(j + 1)) : xc;
        const bool swp = (pat >> j) & 1u;
        if constexpr (UMODE == 2) ustep(std::integral_constant<int, -1>{}, byte_at(j), xc, swp);
        else if (__builtin_expect(swp, 0)) ustep(std::integral_constant<int, 1>{}, byte_at(j), xc, true);
        else ustep(std::integral_constant<int, 0>{}, byte_at(j), xc, false);
        xc = xn;
      }
    }
    else {
      // the node of step j: UMODE 3 from the local-index stream (registers), else
      // through the column-index table in LDS (a dependent read, 2-way bank
      // conflicts between the lane pairs sharing a dword)
      auto node_at = [&](int j) -> int {
        if constexpr (UMODE == 3) return uloc_at(j);
        else return lidx_of(byte_at(j));
      };
      int u1 = node_at(0);
      V3 xc = coord(u1);
      u1 = node_at(1);
#pragma unroll
      for (int j = 0; j < NSTEP; ++j) {
        if ((j & 3) == 0 && j >= nsteps) break;
        const int u2 = j + 2 < NSTEP ? node_at(j + 2) : 0;
        const V3 xn = j + 1 < NSTEP ? coord(u1) : xc;
        step(byte_at(j), xc);
        xc = xn;
        u1 = u2;
      }
    }

    // ---- RHS (unconditional store: idle lanes repeat an active lane's store)
    {
      const unsigned long long am = __ballot(active);
      const int src = active ? lane : (int)__ffsll((long long)am) - 1;
      const double rv = __shfl(f_meas * macc, src);
      const int32_t rr = __shfl(row, src);
      if (rhs) st_out(&rhs[rr], rhs_add ? rhs[rr] + rv : rv);
    }
    wave_sync_lds();

    // ---- diagonal + write-back through a flat LDS image (as k_assemble_p1;
    // the map overlays the coordinates).  (Per-lane 16-B stores straight from
    // registers measured ~2% slower on C2.)
    int fp = len;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(fp, o);
      if (lane >= o) fp += t;
    }
    const int total = __shfl(fp, 63);
    fp -= len;
    uint16_t* map = reinterpret_cast<uint16_t*>(cxyz);
    const uint32_t dsl = active ? dslot : 0xFFu;
    const u32x4 pq = cur.pq;
    if (UNI || PERM || W <= MAXW) {  // canonical structures: W <= 16 = MAXW (sparsity.hip)
      // The diagonal accumulator is zeroed first (on the uniform path it holds
      // the padding steps' sink values): the row sum then runs over all W
      // slots with no per-slot test (slots past the row's end stay 0, and
      // adding +0 changes no bits), and the diagonal (-sum) is written after
      // the row's other values.  The map gives every flat position its value
      // index in `vals` (32 bits: nnz < 2^32, checked on the host).
      if (active) acc_lane[64 * dslot] = 0.0;
      double rv[MAXW];
#pragma unroll
      for (int t = 0; t < MAXW; ++t) rv[t] = acc_lane[64 * min(t, W - 1)];
      double sum = 0.0;
#pragma unroll
      for (int t = 0; t < MAXW; ++t)
        if (t < W) sum += rv[t];  // uniform bound
      uint32_t* const map32 = reinterpret_cast<uint32_t*>(cxyz);
      wave_sync_lds();  // every lane's reads before the overlapping flat writes
#pragma unroll
      for (int t = 0; t < MAXW; ++t)
        if (t < len) {
          acc[fp + t] = rv[t];
          map32[fp + t] = (uint32_t)(rb + (PERM ? pbyte(pq, t) : (uint32_t)t));
        }
      if (active) acc[fp + dslot] = -sum;
      wave_sync_lds();
#pragma unroll
      for (int k = 0; k < MAXW; ++k) {
        const int P = min(64 * k + lane, total - 1);
        st_out(&vals[map32[P]], acc[P]);
      }
    }
    else {
      if (dsl != 0xFFu) {
        double sum = 0.0;
        for (int t = 0; t < len; ++t)
          if (t != (int)dsl) sum += acc_lane[64 * t];
        acc_lane[64 * dsl] = -sum;
      }
      wave_sync_lds();
      for (int t = 0; t < len; ++t) map[fp + t] = (uint16_t)(t * 64 + lane);
      rbs[lane] = rb;
      wave_sync_lds();
      for (int p = lane; p < total; p += 64) {
        const int ix = map[p];
        st_out(&vals[rbs[ix & 63] + (ix >> 6)], acc[ix]);
      }
    }
    wave_sync_lds();
#ifdef AFEM_WAVE_TIMES
    AFEM_WT(2, ++n_done);
#endif
    if (p1 >= r1) break;
    p0 = p1;
    p1 = p2;
    p2 = p3;
    p3 = claim_get(t4);
    R0 = R1;
    R1 = R2;
    R2 = R3;
    if constexpr (USLOT) {
      S0 = S1;
      S1 = S2;
      S2 = S3;
    }
    cur = nxt;
#pragma unroll
    for (int k = 0; k < 4; ++k) nid1[k] = nid2[k];
  }
  AFEM_WT(1, __builtin_amdgcn_s_memrealtime());
}

// ---------------------------------------------------------------- scalar P1, stencil instance
// The uniform slices whose rows all follow ONE strip signature SIG known at
// compile time (StencilSig: steps, shift/swap pattern, slot of every step, row
// length, diagonal slot; matched byte for byte by the structure build,
// stencil_match): the interior bricks of a structured box, 97.5 % of the C2
// slices.  With the slots constant, the row's accumulators are REGISTERS
// (acc[W], indexed by compile-time window slots): no LDS accumulators, no
// ds_add_f64 in the step loop, no zero fill, no scalar shift/swap branches,
// no slot stream; the LDS holds the slice's coordinates and, after the steps,
// the write-back image (position P = lane * W + t: no map, the value index is
// rbs[P / W] + P % W).  Arithmetic, entry by entry, in the uniform instance's
// order (each accumulator starts at +0 and adds the steps' products in step
// order, rounded like ds_add_f64: the adds are not contracted): the three
// instances give the same bits.
#include "stencil_sigs.inc"  // constexpr StencilSig kSig<name> (StencilSig: afem_internal.hpp)
#define AFEM_STENCIL_PTR(ID_, SIG_) &SIG_,
inline constexpr const StencilSig* kStencilSigPtrs[] = { AFEM_STENCIL_SIGS(AFEM_STENCIL_PTR) };
#undef AFEM_STENCIL_PTR

template <const StencilSig& S>
struct StencilWin {  // slots of the window nodes P, Q, R after step j's rotation
  int p[32] = {}, q[32] = {}, r[32] = {};
  // first[j]: the node step j drops leaves the window for the first time (its
  // accumulator's first contribution: a store, not an add); fin[k]: the same for
  // the final P, Q, R
  bool first[32] = {}, fin[3] = {};
  constexpr StencilWin()
  {
    bool seen[64] = {};
    int P = S.dslot, Q = S.slot[0] & 63, R = S.slot[1] & 63;
    for (int j = 2; j < S.nsteps; ++j) {
      const int d = ((S.pat >> j) & 1u) ? Q : P;
      first[j] = !seen[d];
      seen[d] = true;
      if (!((S.pat >> j) & 1u)) P = Q;
      Q = R;
      R = S.slot[j] & 63;
      p[j] = P;
      q[j] = Q;
      r[j] = R;
    }
    fin[0] = !seen[P];
    seen[P] = true;
    fin[1] = !seen[Q];
    seen[Q] = true;
    fin[2] = !seen[R];
  }
};
template <const StencilSig& S>
inline constexpr StencilWin<S> kStencilWin{};

__device__ __forceinline__ double add_nc(double a, double b)
{
#pragma clang fp contract(off)
  return a + b;  // rounded on its own, as the LDS accumulator's ds_add_f64
}

__host__ __device__ constexpr int64_t stencil_tile_bytes(int64_t u_cap, int64_t w)
{
  // coordinates (24 B per node) overlaid by the write-back image (64 w values), + 64 row offsets
  return ((24 * u_cap > 512 * w ? 24 * u_cap : 512 * w) + 15) / 16 * 16 + 512;
}

// one slice of signature S (the steps, the RHS and the write-back of k_assemble_stencil)
template <const StencilSig& S, int MAXC, bool PERM>
__device__ __forceinline__ void stencil_slice(const StripPre<MAXC>& cur, int nsteps, int lane, const double* cxyz,
                                              double* flat, int64_t* rbs, double s_coef, double f_meas,
                                              double* __restrict__ vals, double* __restrict__ rhs, int rhs_add)
{
  constexpr int W = S.w, D = S.dslot, NS = S.nsteps;
  static_assert(NS <= 16 * MAXC && W <= 16, "stencil signature beyond the kernel's strip chunks");
    const int32_t row = cur.row;
    const bool active = row >= 0;
    auto coord = [&](int u) {
      const double* q = cxyz + 3 * u;
      return V3{ q[0], q[1], q[2] };
    };
    auto uloc_at = [&](int j) -> int {
      const u32x4 w = cur.cu[j >> 4];
      const int q = (j >> 2) & 3;
      const uint32_t wq = q == 0 ? w.x : (q == 1 ? w.y : (q == 2 ? w.z : w.w));
      return (int)((wq >> (8 * (j & 3))) & 0xFFu);
    };
    const V3 xi = coord((int)(cur.dl >> 16));
    double acc[W];
#pragma unroll
    for (int t = 0; t < W; ++t) acc[t] = 0.0;
    double macc = 0.0;
    V3 eP{ 0.0, 0.0, 0.0 }, eQ = sub(coord(uloc_at(0)), xi), eR = sub(coord(uloc_at(1)), xi);
    V3 cP = cross(eQ, eR), cN{ 0.0, 0.0, 0.0 };
    V3 xc = coord(uloc_at(2));
    // the uniform instance's loop shape: a scalar guard every 2 steps (the
    // slice's step count, NS for every slice of the list) keeps the steps in
    // their own blocks, so the coordinate reads stay one step ahead instead of
    // being hoisted all at once; after full unrolling the window slots and the
    // shift/swap arms are constants
#pragma unroll
    for (int j = 2; j < NS; ++j) {
      if ((j & 1) == 0 && j >= nsteps) break;
      const V3 xn = j + 1 < NS ? coord(uloc_at(j + 1 < NS ? j + 1 : j)) : xc;
      const V3 eD = sub(xc, xi);
      V3 cRn;
      if ((S.pat >> j) & 1u) {
        cRn = cN;
      }
      else {
        cRn = cP;
        eP = eQ;
      }
      eQ = eR;
      eR = eD;
      cP = cross(eQ, eR);
      cN = cross(eP, eR);
      const V3 m = V3{ cP.x - cN.x + cRn.x, cP.y - cN.y + cRn.y, cP.z - cN.z + cRn.z };
      const double meas = fabs(dot(eP, cP));
      const double s = -s_coef * recip1(meas);  // no padding steps run here: meas > 0
      const double kP = dot(m, cP) * s;
      const double kQ = -dot(m, cN) * s;
      const double kR = dot(m, cRn) * s;
      macc += meas;
      const int iP = kStencilWin<S>.p[j], iQ = kStencilWin<S>.q[j], iR = kStencilWin<S>.r[j];
      acc[iP] = add_nc(acc[iP], kP);
      acc[iQ] = add_nc(acc[iQ], kQ);
      acc[iR] = add_nc(acc[iR], kR);
      // keep the adds in their step: an accumulator read only at the end would
      // otherwise be summed there (machine sinking), with all 3 x 24 products live
      asm volatile("" : "+v"(acc[iP]), "+v"(acc[iQ]), "+v"(acc[iR]));
      xc = xn;
    }

    // ---- RHS (as k_assemble_strip)
    {
      const unsigned long long am = __ballot(active);
      const int src = active ? lane : (int)__ffsll((long long)am) - 1;
      const double rv = __shfl(f_meas * macc, src);
      const int32_t rr = __shfl(row, src);
      if (rhs) st_out(&rhs[rr], rhs_add ? rhs[rr] + rv : rv);
    }
    // ---- diagonal (-sum of the row's other entries, in slot order) + write-back image
    double sum = 0.0;
#pragma unroll
    for (int t = 0; t < W; ++t)
      if (t != D) sum += acc[t];
    // brick x-runs: when lanes 4q..4q+3 hold consecutive rows (all of the
    // signature's length W), their 4W values are one contiguous range at rb(4q):
    // the run's base is a wave-uniform scalar and lane l stores value l of the
    // run -- no owner division, no dependent LDS read of the row offsets
    const int64_t rb = active ? cur.rb : -1;
    const int64_t rb_run = __shfl(rb, lane & ~3);
    // (canonical structures store through the slot map: no runs)
    const bool runs = !PERM && __all(active && rb == rb_run + (int64_t)W * (lane & 3));
    if constexpr (PERM) {
      // canonical structure: the rows are scattered over the matrix (the
      // caller's numbering), so a lane's own W stores would touch 64 rows per
      // instruction.  Row L's values go to flat positions [W L, W (L + 1)) at
      // their physical slots (the slot map), then consecutive lanes store
      // consecutive positions: W / 64 rows per instruction, each row's values
      // one contiguous range (the flat image of k_assemble_strip)
      wave_sync_lds();  // every lane's coordinate reads before the image overwrites them
#pragma unroll
      for (int t = 0; t < W; ++t) flat[lane * W + (int)pbyte(cur.pq, t)] = t == D ? -sum : acc[t];
      rbs[lane] = rb;
      wave_sync_lds();
#pragma unroll
      for (int k = 0; k < W; ++k) {
        const int P = 64 * k + lane;
        const int L = P / W;  // constant divisor
        const int64_t base = rbs[L];
        if (base >= 0) st_out(&vals[base + (P - L * W)], flat[P]);
      }
    }
    else if (runs) {
      static_assert(4 * W <= 64, "a run's values exceed the wave");
      wave_sync_lds();  // every lane's coordinate reads before the image overwrites them
#pragma unroll
      for (int t = 0; t < W; ++t) flat[lane * W + t] = t == D ? -sum : acc[t];
      wave_sync_lds();
      // lanes past the run's 4W values repeat its last value (same address, same
      // value): no exec-mask branch, so the 16 image reads issue together
      const int o = lane < 4 * W ? lane : 4 * W - 1;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)rb, 4 * r);
        const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)rb >> 32), 4 * r);
        double* const dst = vals + (int64_t)(((uint64_t)hi << 32) | lo);
        st_out(&dst[o], flat[4 * W * r + o]);
      }
    }
    else if (active) {
      // partial bricks and face tiles whose lanes are not x-runs (a few % of the
      // slices): each lane stores its row's W values straight from the registers
      // (no image, no owner table: nothing of this path is kept live across slices)
#pragma unroll
      for (int t = 0; t < W; ++t) st_out(&vals[rb + t], t == D ? -sum : acc[t]);
    }
    wave_sync_lds();
}

// signature index -> stencil_slice<S_index> (a scalar branch per slice)
template <bool PERM, int I, const StencilSig& S0, const StencilSig&... SR>
struct StencilDispatch {
  template <int MAXC>
  __device__ __forceinline__ static void run(int sig, const StripPre<MAXC>& cur, int nsteps, int lane,
                                             const double* cxyz, double* flat, int64_t* rbs, double s_coef,
                                             double f_meas, double* vals, double* rhs, int rhs_add)
  {
    if (sig == I || sizeof...(SR) == 0)
      stencil_slice<S0, MAXC, PERM>(cur, nsteps, lane, cxyz, flat, rbs, s_coef, f_meas, vals, rhs, rhs_add);
    else if constexpr (sizeof...(SR) > 0)
      StencilDispatch<PERM, I + 1, SR...>::template run<MAXC>(sig, cur, nsteps, lane, cxyz, flat, rbs, s_coef, f_meas,
                                                        vals, rhs, rhs_add);
  }
};

template <const StencilSig&... SS>
constexpr int stencil_maxc()
{
  int m = 1;
  for (int c : { ((SS.nsteps + 15) / 16)... }) m = c > m ? c : m;
  return m;
}
template <const StencilSig&... SS>
constexpr int stencil_maxw()
{
  int m = 1;
  for (int w : { SS.w... }) m = w > m ? w : m;
  return m;
}

template <bool PERM, const StencilSig&... SS>
__global__ __launch_bounds__(64, 2) void k_assemble_stencil(int64_t n_slices, const SliceRec* __restrict__ recs,
                                                            unsigned long long* __restrict__ tickets, int u_cap,
                                                            const int32_t* __restrict__ perm,
                                                            const int64_t* __restrict__ pos_rb,
                                                            const uint32_t* __restrict__ pos_dl,
                                                            const uint8_t* __restrict__ strip_u,
                                                            const int32_t* __restrict__ snode,
                                                            const double* __restrict__ coords, double s_coef,
                                                            double f_meas, double* __restrict__ vals,
                                                            double* __restrict__ rhs, int rhs_add,
                                                            const uint8_t* __restrict__ cperm)
{
  constexpr int MAXC = stencil_maxc<SS...>();
  extern __shared__ __align__(16) unsigned char smem[];
  double* const cxyz = reinterpret_cast<double*>(smem);
  double* const flat = cxyz;  // the write-back image overlays the coordinates
  int64_t* const rbs = reinterpret_cast<int64_t*>(smem + stencil_tile_bytes(u_cap, stencil_maxw<SS...>()) - 512);
  const int lane = threadIdx.x;
  // claiming and the four-stage pipeline of k_assemble_strip
  const int xcd = (int)(blockIdx.x & 7);
  const int64_t r0 = n_slices * xcd / 8, r1 = n_slices * (xcd + 1) / 8;
  auto claim_issue = [&]() -> unsigned long long {
    unsigned long long t = 0;
    if (lane == 0) t = atomicAdd(tickets + 16 * xcd, 1ull);
    return t;
  };
  auto claim_get = [&](unsigned long long t) -> int64_t {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)t);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(t >> 32));
    return r0 + (int64_t)(((uint64_t)hi << 32) | lo);
  };
  int64_t p0 = claim_get(claim_issue());
  if (p0 >= r1) return;
  int64_t p1 = claim_get(claim_issue());
  int64_t p2 = claim_get(claim_issue());
  int64_t p3 = claim_get(claim_issue());
  SliceRec R0 = recs[p0];
  SliceRec R1 = recs[p1 < r1 ? p1 : p0];
  SliceRec R2 = recs[p2 < r1 ? p2 : p0];
  auto load_nid = [&](const SliceRec& R, int32_t(&nid)[4]) {
    const int nu = (int)(R.meta & 0xFFFFu);
#pragma unroll
    for (int k = 0; k < 4; ++k) nid[k] = snode[(int64_t)R.snode_off + max(min(lane + 64 * k, nu - 1), 0)];
  };
  auto load_rows = [&](const SliceRec& R, StripPre<MAXC>& p) {
    const int64_t q = (int64_t)R.sl * 64 + lane;
    p.row = perm[q];
    p.dl = pos_dl[q];
    p.rb = pos_rb[q];
    if constexpr (PERM) p.pq = reinterpret_cast<const u32x4*>(cperm)[q];
    const u32x4* su = reinterpret_cast<const u32x4*>(strip_u + (int64_t)R.strip_off * 1024) + lane;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) p.cu[c] = su[(int64_t)c * 64];
  };
  auto gather = [&](const int32_t(&nid)[4], StripPre<MAXC>& p) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      p.x[k] = coords[3 * (int64_t)nid[k]];
      p.y[k] = coords[3 * (int64_t)nid[k] + 1];
      p.z[k] = coords[3 * (int64_t)nid[k] + 2];
    }
  };
  StripPre<MAXC> cur, nxt;
  int32_t nid1[4], nid2[4];
  {
    int32_t nid0[4];
    load_nid(R0, nid0);
    load_rows(R0, cur);
    gather(nid0, cur);
    load_nid(R1, nid1);
  }
  __builtin_amdgcn_s_waitcnt(0);
  for (;;) {
    const unsigned long long t4 = claim_issue();
    const SliceRec R3 = recs[p3 < r1 ? p3 : p0];
    const int nu = (int)(R0.meta & 0xFFFFu);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int idx = max(min(lane + 64 * k, nu - 1), 0);
      cxyz[3 * idx] = cur.x[k];
      cxyz[3 * idx + 1] = cur.y[k];
      cxyz[3 * idx + 2] = cur.z[k];
    }
    wave_sync_lds();
    load_rows(R1, nxt);
    gather(nid1, nxt);
    load_nid(R2, nid2);

    StencilDispatch<PERM, 0, SS...>::template run<MAXC>((int)R0.sig, cur, (int)(R0.meta >> 24), lane, cxyz, flat, rbs,
                                                  s_coef, f_meas, vals, rhs, rhs_add);
    if (p1 >= r1) break;
    p0 = p1;
    p1 = p2;
    p2 = p3;
    p3 = claim_get(t4);
    R0 = R1;
    R1 = R2;
    R2 = R3;
    cur = nxt;
#pragma unroll
    for (int k = 0; k < 4; ++k) nid1[k] = nid2[k];
  }
}

// Shared factors of a step's three window blocks (rotated frame: component
// row x; c_row = -m, the sign folded into s < 0):
//   K_rb^{00} = s [(lambda + 2 mu) m_x c_x + mu m_y c_y + mu m_z c_z] + mass
//   K_rb^{01} = s [lambda m_x c_y + mu m_y c_x],  K_rb^{02} = s [lambda m_x c_z + mu m_z c_x]
// with the scale folded into four per-step factors A = s (lambda + 2 mu) m_x,
// B = s mu m_y, C = s mu m_z, D = s lambda m_x (7 FP64 operations per step):
// per block then 3 + 2 + 2 fused multiply-adds and one add (the mass), the
// accumulation included -- 8 operations instead of 12.  (A uniform padding
// step's huge s meets finite m: the factors stay finite, and they only feed
// the diagonal slot's sink.)
struct ElastPre {
  double A, B, C, D;
};
// kernel constants: the 1/6 of the element scale 1/(6|det|) and the mass
// factor c0/120 folded in once (s = -1/|det| per step)
struct ElastK {
  double a, b, d, m120;
};
__device__ __forceinline__ ElastK elast_consts(double lambda, double mu, double c0)
{
  return ElastK{ (lambda + 2.0 * mu) * (1.0 / 6.0), mu * (1.0 / 6.0), lambda * (1.0 / 6.0), c0 * (1.0 / 120.0) };
}
__device__ __forceinline__ ElastPre elast_pre(V3 m, double s, const ElastK& k)
{
  const double sx = s * m.x, sy = s * m.y, sz = s * m.z;
  return ElastPre{ k.a * sx, k.b * sy, k.b * sz, k.d * sx };
}
// explicit fma throughout: one rounding sequence whatever the instance (the
// uniform and general instances, the one-wave and workgroup kernels agree bit
// for bit)
__device__ __forceinline__ void elast_block(double* a, const ElastPre& e, V3 c, double mass)
{
  atomicAdd(a, fma(e.A, c.x, fma(e.B, c.y, fma(e.C, c.z, mass))));
  atomicAdd(a + 64, fma(e.D, c.y, e.B * c.x));
  atomicAdd(a + 128, fma(e.D, c.z, e.C * c.x));
}
// the same three entries added to register partial sums g (register-window
// accumulation)
__device__ __forceinline__ V3 elast_acc(V3 g, const ElastPre& e, V3 c, double mass)
{
  return V3{ fma(e.A, c.x, fma(e.B, c.y, fma(e.C, c.z, add_nc(g.x, mass)))), fma(e.D, c.y, fma(e.B, c.x, g.y)),
             fma(e.D, c.z, fma(e.C, c.x, g.z)) };
}
// a node's first step in the window (its partial sums start here)
__device__ __forceinline__ V3 elast_first(const ElastPre& e, V3 c, double mass)
{
  return V3{ fma(e.A, c.x, fma(e.B, c.y, fma(e.C, c.z, mass))), fma(e.D, c.y, e.B * c.x), fma(e.D, c.z, e.C * c.x) };
}
// flush a window node's register partial sums into its LDS accumulators [k][lane] (stride 64)
__device__ __forceinline__ void flush3(double* a, V3 g)
{
  atomicAdd(a, g.x);
  atomicAdd(a + 64, g.y);
  atomicAdd(a + 128, g.z);
}
// the node's first flush (stencil instance: known at compile time): a store,
// so the accumulators need no zero fill (0 + g = g)
__device__ __forceinline__ void store3(double* a, V3 g)
{
  a[0] = g.x;
  a[64] = g.y;
  a[128] = g.z;
}

// ---------------------------------------------------------------- block-3 elasticity, persistent strips
// k_assemble_elast_tet restructured like k_assemble_strip: persistent waves
// claim work items (slice, component row ci) per XCD (the three items of a
// slice are adjacent: one L2 serves their shared coordinates), the same
// four-stage prefetch pipeline over 32-B slice records, and a write-back
// through a flat LDS image (per-row layout: the 3*len values of (row, ci)
// are contiguous; per-block layout: runs of 3).  The wave works in a frame
// whose axes are cyclically rotated by ci (coordinates staged as
// (x_ci, x_ci+1, x_ci+2)): its component row is always "x", no per-step
// component selects; value (t, k) of the rotated frame is column
// (ci + k) % 3 of the block.  A cyclic axis permutation is a rotation, the
// material isotropic: the entries are the same numbers (up to the order of
// the three products in a dot product).
// BIG: unstructured meshes (rows up to 32 slots, slices of more than 256
// nodes, strips up to 64 steps): the nodes past the first 256 and the
// column-index entries past the first 128 words are staged straight from
// memory, and the write-back stores each lane's values directly (two passes
// over the accumulators: diagonal sums, then values) instead of holding 3 x
// MAXW values in registers for the flat image.
template <int MAXC, int MAXW, int UMODE, bool BIG = false>
__global__ __launch_bounds__(64) void k_assemble_elast_strip(int64_t n_items, const SliceRec* __restrict__ recs,
                                                             unsigned long long* __restrict__ tickets, int u_cap,
                                                             int w_cap, bool per_block,
                                                             const int32_t* __restrict__ perm,
                                                             const int64_t* __restrict__ pos_rb,
                                                             const uint32_t* __restrict__ pos_dl,
                                                             const uint8_t* __restrict__ strip,
                                                             const uint16_t* __restrict__ lidx,
                                                             const int32_t* __restrict__ snode,
                                                             const double* __restrict__ coords, double lambda,
                                                             double mu, double c0, double fx, double fy, double fz,
                                                             double* __restrict__ vals, double* __restrict__ rhs, int rhs_add)
{
  const ElastK ek = elast_consts(lambda, mu, c0);
  extern __shared__ __align__(16) unsigned char smem[];
  double* acc = reinterpret_cast<double*>(smem);  // [slot][k][lane]
  double* cxyz = reinterpret_cast<double*>(smem + 3 * 8 * 64 * (int64_t)w_cap);
  const int64_t cbytes = elast_coord_bytes(u_cap, w_cap);
  uint16_t* li = reinterpret_cast<uint16_t*>(reinterpret_cast<unsigned char*>(cxyz) + cbytes);
  int64_t* rbs = reinterpret_cast<int64_t*>(reinterpret_cast<unsigned char*>(li) + 2 * 64 * (int64_t)w_cap);
  const int lane = threadIdx.x;
  const int xcd = (int)(blockIdx.x & 7);
  const int64_t r0 = n_items * xcd / 8, r1 = n_items * (xcd + 1) / 8;
  auto claim_issue = [&]() -> unsigned long long {
    unsigned long long t = 0;
    if (lane == 0) t = atomicAdd(tickets + 16 * xcd, 1ull);
    return t;
  };
  auto claim_get = [&](unsigned long long t) -> int64_t {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)t);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(t >> 32));
    return r0 + (int64_t)(((uint64_t)hi << 32) | lo);
  };
  int64_t p0 = claim_get(claim_issue());
  if (p0 >= r1) return;
  int64_t p1 = claim_get(claim_issue());
  int64_t p2 = claim_get(claim_issue());
  int64_t p3 = claim_get(claim_issue());
  SliceRec R0 = recs[p0 / 3];
  SliceRec R1 = recs[(p1 < r1 ? p1 : p0) / 3];
  SliceRec R2 = recs[(p2 < r1 ? p2 : p0) / 3];

  auto load_nid = [&](const SliceRec& R, int32_t(&nid)[4]) {
    const int nu = (int)(R.meta & 0xFFFFu);
#pragma unroll
    for (int k = 0; k < 4; ++k) nid[k] = snode[(int64_t)R.snode_off + max(min(lane + 64 * k, nu - 1), 0)];
  };
  auto load_rows = [&](const SliceRec& R, StripPre<MAXC>& p) {
    const int64_t q = (int64_t)R.sl * 64 + lane;
    p.row = perm[q];
    p.dl = pos_dl[q];
    p.rb = pos_rb[q];
    const int nq = 8 * (int)((R.meta >> 16) & 0xFFu);
    const u32x4* ls = reinterpret_cast<const u32x4*>(lidx + R.lidx_off);
    p.l0 = ls[max(min(lane, nq - 1), 0)];
    p.l1 = ls[max(min(lane + 64, nq - 1), 0)];
    const int nc = (int)((R.meta >> 24) + 15) >> 4;
    const u32x4* sp = reinterpret_cast<const u32x4*>(strip + (int64_t)R.strip_off * 1024) + lane;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) p.ch[c] = sp[(int64_t)max(min(c, nc - 1), 0) * 64];
  };
  auto gather = [&](const int32_t(&nid)[4], StripPre<MAXC>& p) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      p.x[k] = coords[3 * (int64_t)nid[k]];
      p.y[k] = coords[3 * (int64_t)nid[k] + 1];
      p.z[k] = coords[3 * (int64_t)nid[k] + 2];
    }
  };
  StripPre<MAXC> cur, nxt;
  int32_t nid1[4], nid2[4];
  {
    int32_t nid0[4];
    load_nid(R0, nid0);
    load_rows(R0, cur);
    gather(nid0, cur);
    load_nid(R1, nid1);
  }
  __builtin_amdgcn_s_waitcnt(0);
  for (;;) {
    const unsigned long long t4 = claim_issue();
    const SliceRec R3 = recs[(p3 < r1 ? p3 : p0) / 3];
    const int ci = (int)(p0 % 3);  // component row (uniform)
    const int nsteps = (int)(R0.meta >> 24);
    const int W = (int)((R0.meta >> 16) & 0xFFu);
    const int nu = (int)(R0.meta & 0xFFFFu);
    // ---- stage: coordinates in the rotated frame, column indices, zero accumulators
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int idx = max(min(lane + 64 * k, nu - 1), 0);
      const double a = cur.x[k], b = cur.y[k], c = cur.z[k];
      cxyz[3 * idx] = ci == 0 ? a : (ci == 1 ? b : c);
      cxyz[3 * idx + 1] = ci == 0 ? b : (ci == 1 ? c : a);
      cxyz[3 * idx + 2] = ci == 0 ? c : (ci == 1 ? a : b);
    }
    if (BIG && nu > 256) {
      for (int u = lane + 256; u < nu; u += 64) {
        const int64_t nd = snode[(int64_t)R0.snode_off + u];
        const double a = coords[3 * nd], b = coords[3 * nd + 1], c = coords[3 * nd + 2];
        cxyz[3 * u] = ci == 0 ? a : (ci == 1 ? b : c);
        cxyz[3 * u + 1] = ci == 0 ? b : (ci == 1 ? c : a);
        cxyz[3 * u + 2] = ci == 0 ? c : (ci == 1 ? a : b);
      }
    }
    {
      const int nq = 8 * W;
      u32x4* dst = reinterpret_cast<u32x4*>(li);
      dst[max(min(lane, nq - 1), 0)] = cur.l0;
      dst[max(min(lane + 64, nq - 1), 0)] = cur.l1;
      if (BIG && nq > 128) {
        const u32x4* ls = reinterpret_cast<const u32x4*>(lidx + R0.lidx_off);
        for (int q = lane + 128; q < nq; q += 64) dst[q] = ls[q];
      }
      double2* a2 = reinterpret_cast<double2*>(acc);
      for (int q = lane; q < 96 * W; q += 64) a2[q] = make_double2(0.0, 0.0);
    }
    wave_sync_lds();
    load_rows(R1, nxt);
    gather(nid1, nxt);
    load_nid(R2, nid2);

    const int32_t row = cur.row;
    const bool active = row >= 0;
    const int64_t rb = cur.rb;
    const int len = (int)((cur.dl >> 8) & 0xFFu);
    const uint32_t dslot = cur.dl & 0xFFu;
    const uint16_t* lrow = li + lane;
    const V3 xi = [&] {
      const double* q = cxyz + 3 * (int)lrow[dslot * 64];
      return V3{ q[0], q[1], q[2] };
    }();
    double macc = 0.0;
    V3 eP{ 0.0, 0.0, 0.0 }, eQ{ 0.0, 0.0, 0.0 }, eR{ 0.0, 0.0, 0.0 };
    V3 cP{ 0.0, 0.0, 0.0 }, cN{ 0.0, 0.0, 0.0 };
    double* const acc_lane = acc + lane;
    double* aP = acc_lane + 192 * dslot;
    double* aQ = aP;
    double* aR = aP;
    auto lidx_of = [&](uint32_t byte) { return (int)lrow[(byte & 63u) * 64]; };
    auto coord = [&](int u) {
      const double* q = cxyz + 3 * u;
      return V3{ q[0], q[1], q[2] };
    };
    auto sel = [](bool c, V3 a, V3 b) { return V3{ c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z }; };
    auto keep = [](uint64_t m, double x) { return __longlong_as_double((long long)(m & (uint64_t)__double_as_longlong(x))); };
    // entries (0, k) of K_rb in the rotated frame, c_r = -m (sign folded into s < 0)
    auto block = [&](double* a, const ElastPre& e, V3 cb, double mass) { elast_block(a, e, cb, mass); };
    auto step = [&](uint32_t byte, V3 xd) {
      const bool swap = (byte & 0xC0u) == 0x40u;
      const uint64_t em = (uint64_t)0 - (uint64_t)(byte < 0x80u);
      double* const aD = acc_lane + 192 * (byte & 63u);
      const V3 eD = sub(xd, xi);
      const V3 cRn = sel(swap, cN, cP);
      eP = sel(swap, eP, eQ);
      aP = swap ? aP : aQ;
      eQ = eR;
      aQ = aR;
      eR = eD;
      aR = aD;
      cP = cross(eQ, eR);
      cN = cross(eP, eR);
      const V3 m = V3{ cP.x - cN.x + cRn.x, cP.y - cN.y + cRn.y, cP.z - cN.z + cRn.z };
      const double meas = fabs(dot(eP, cP));
      const double s = keep(em, -recip1(meas));
      const double mass = keep(em, meas * ek.m120);
      macc += keep(em, meas);
      const ElastPre e = elast_pre(m, s, ek);
      block(aP, e, cP, mass);
      block(aQ, e, V3{ -cN.x, -cN.y, -cN.z }, mass);
      block(aR, e, cRn, mass);
    };
    auto byte_at = [&](int j) -> uint32_t {
      const u32x4 w = cur.ch[j >> 4];
      const int q = (j >> 2) & 3;
      const uint32_t wq = q == 0 ? w.x : (q == 1 ? w.y : (q == 2 ? w.z : w.w));
      return (wq >> (8 * (j & 3))) & 0xFFu;
    };
    constexpr int NSTEP = 16 * MAXC;
    if constexpr (UMODE == 1) {
      // uniform slice (as k_assemble_strip<.., 1>): priming steps only load
      // the window, scalar shift/swap branches, no emit masks; a padding step
      // (odd lengths) has a zero edge and only feeds the diagonal slot
      const uint64_t pat = R0.pat;
      auto ustep = [&](auto swap_c, uint32_t byte, V3 xd) {
        constexpr bool SWAP = decltype(swap_c)::value;
        double* const aD = acc_lane + 192 * (byte & 63u);
        const V3 eD = sub(xd, xi);
        V3 cRn;
        if constexpr (SWAP) {
          cRn = cN;
        }
        else {
          cRn = cP;
          eP = eQ;
          aP = aQ;
        }
        eQ = eR;
        aQ = aR;
        eR = eD;
        aR = aD;
        cP = cross(eQ, eR);
        cN = cross(eP, eR);
        const V3 m = V3{ cP.x - cN.x + cRn.x, cP.y - cN.y + cRn.y, cP.z - cN.z + cRn.z };
        const double meas = fabs(dot(eP, cP));
        const double s = -recip1(fmax(meas, 1e-300));
        const double mass = meas * ek.m120;
        macc += meas;
        const ElastPre e = elast_pre(m, s, ek);
        block(aP, e, cP, mass);
        block(aQ, e, V3{ -cN.x, -cN.y, -cN.z }, mass);
        block(aR, e, cRn, mass);
      };
      {
        const uint32_t b0 = byte_at(0), b1 = byte_at(1);
        eQ = sub(coord(lidx_of(b0)), xi);
        eR = sub(coord(lidx_of(b1)), xi);
        aQ = acc_lane + 192 * (b0 & 63u);
        aR = acc_lane + 192 * (b1 & 63u);
        cP = cross(eQ, eR);
      }
      int u1 = lidx_of(byte_at(2));
      V3 xc = coord(u1);
      u1 = lidx_of(byte_at(3));
#pragma unroll
      for (int j = 2; j < NSTEP; ++j) {
        if ((j & 1) == 0 && j >= nsteps) break;
        const int u2 = j + 2 < NSTEP ? lidx_of(byte_at(j + 2)) : 0;
        const V3 xn = j + 1 < NSTEP ? coord(u1) : xc;
        if (__builtin_expect((pat >> j) & 1u, 0)) ustep(std::true_type{}, byte_at(j), xc);
        else ustep(std::false_type{}, byte_at(j), xc);
        xc = xn;
        u1 = u2;
      }
    }
    else {
      int u1 = lidx_of(byte_at(0));
      V3 xc = coord(u1);
      u1 = lidx_of(byte_at(1));
#pragma unroll
      for (int j = 0; j < NSTEP; ++j) {
        if ((j & 3) == 0 && j >= nsteps) break;
        const int u2 = j + 2 < NSTEP ? lidx_of(byte_at(j + 2)) : 0;
        const V3 xn = j + 1 < NSTEP ? coord(u1) : xc;
        step(byte_at(j), xc);
        xc = xn;
        u1 = u2;
      }
    }
    if (rhs && active) {
    const double rv = (ci == 0 ? fx : (ci == 1 ? fy : fz)) * macc * (1.0 / 24.0);
    st_out(&rhs[3 * (int64_t)row + ci], rhs_add ? rhs[3 * (int64_t)row + ci] + rv : rv);
  }
    wave_sync_lds();

    if constexpr (BIG) {
      // ---- diagonal block row (sums over the row's slots), then direct stores
      if (active) {
        acc_lane[192 * dslot] = 0.0;
        acc_lane[192 * dslot + 64] = 0.0;
        acc_lane[192 * dslot + 128] = 0.0;
      }
      double sum[3] = { 0.0, 0.0, 0.0 };
      for (int t = 0; t < W; ++t)  // slots past the row's end hold 0
#pragma unroll
        for (int k = 0; k < 3; ++k) sum[k] += acc_lane[192 * t + 64 * k];
      if (active) {
        for (int t = 0; t < len; ++t) {
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            const int j = k + ci < 3 ? k + ci : k + ci - 3;
            const double v =
                t == (int)dslot ? add_nc(-sum[k], k == 0 ? c0 * macc * (1.0 / 24.0) : 0.0) : acc_lane[192 * t + 64 * k];
            st_out(&vals[per_block ? 9 * (rb + t) + 3 * ci + j : 9 * rb + 3 * (int64_t)ci * len + 3 * t + j], v);
          }
        }
      }
    }
    else {
    // ---- diagonal block row + write-back through a flat LDS image
    // (3*len values per lane; map: position -> lane | offset << 6 with the
    // value index = rbs[lane] + offset: per block 9 rb + 3 ci + (9 t + j),
    // per row 9 rb + 3 ci len + (3 t + j))
    const int n3 = 3 * len;
    int fp = n3;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(fp, o);
      if (lane >= o) fp += t;
    }
    const int total = __shfl(fp, 63);
    fp -= n3;
    if (active) {
      acc_lane[192 * dslot] = 0.0;
      acc_lane[192 * dslot + 64] = 0.0;
      acc_lane[192 * dslot + 128] = 0.0;
    }
    double rv[3 * MAXW];
#pragma unroll
    for (int t = 0; t < MAXW; ++t)
#pragma unroll
      for (int k = 0; k < 3; ++k) rv[3 * t + k] = acc_lane[192 * min(t, W - 1) + 64 * k];
    double sum[3] = { 0.0, 0.0, 0.0 };
#pragma unroll
    for (int t = 0; t < MAXW; ++t)
      if (t < W)
#pragma unroll
        for (int k = 0; k < 3; ++k) sum[k] += rv[3 * t + k];
    uint16_t* map = reinterpret_cast<uint16_t*>(cxyz);
    wave_sync_lds();  // every lane's reads before the overlapping flat writes
#pragma unroll
    for (int t = 0; t < MAXW; ++t)
      if (t < len) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          // value (t, k) of the rotated frame = block column (ci + k) % 3
          const int j = k + ci < 3 ? k + ci : k + ci - 3;
          acc[fp + 3 * t + j] = rv[3 * t + k];
          map[fp + 3 * t + j] = (uint16_t)(lane | (per_block ? 9 * t + j : 3 * t + j) << 6);
        }
      }
    if (active) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int j = k + ci < 3 ? k + ci : k + ci - 3;
        acc[fp + 3 * (int)dslot + j] = add_nc(-sum[k], k == 0 ? c0 * macc * (1.0 / 24.0) : 0.0);
      }
    }
    rbs[lane] = 9 * rb + 3 * ci * (per_block ? 1 : (int64_t)len);
    wave_sync_lds();
    for (int k = 0; k < 3 * MAXW; ++k) {
      if (64 * k >= total) break;  // uniform
      const int Pc = min(64 * k + lane, total - 1);
      const int m = map[Pc];
      st_out(&vals[rbs[m & 63] + (m >> 6)], acc[Pc]);
    }
    }
    wave_sync_lds();
    if (p1 >= r1) break;
    p0 = p1;
    p1 = p2;
    p2 = p3;
    p3 = claim_get(t4);
    R0 = R1;
    R1 = R2;
    R2 = R3;
    cur = nxt;
#pragma unroll
    for (int k = 0; k < 4; ++k) nid1[k] = nid2[k];
  }
}

// ---------------------------------------------------------------- block-3 elasticity, one workgroup per slice
// k_assemble_elast_strip with the three component rows of a slice in ONE
// workgroup of three waves (wave i = component row i): the slice's node
// coordinates (SoA, bank-aware positions) and column-index table are staged
// once for the three waves (one global gather per slice instead of three),
// and the write-back goes through one flat LDS image of the slice's
// complete 3x3 blocks (per block 9 contiguous values, per row 9 len): the
// workgroup stores whole blocks with consecutive threads (no 24-B pieces
// of 72-B blocks from three different waves: WRITE_SIZE was 1.3x the
// values).  LDS per workgroup: 3 x [slot][3][lane] accumulators (the flat
// image overlays them) + coordinates + column indices: 2 workgroups = 6
// waves per CU (the one-wave-per-item kernel: 5).  Coordinates are read in
// the frame rotated by the wave's component row (three SoA reads at
// rotated array offsets), so the element arithmetic is that of
// k_assemble_elast_strip, entry for entry.
// the stencil instance's full-slice x-run stores: 16 B per thread
// (AFEM_WG_ST16=0 builds the 8-B stores, for A/B)
#ifndef AFEM_WG_ST16
#define AFEM_WG_ST16 1
#endif
// the stencil instance's x-run stores non-temporal (the values are not re-read by the launch; C3
// 1.72 -> 1.68 ms median, r05bn, tools/ab_lib.py against a -DAFEM_WG_NT=0 build)
#ifndef AFEM_WG_NT
#define AFEM_WG_NT 1
#endif
__host__ __device__ constexpr int64_t elast_wg_bytes(int64_t u_cap, int64_t w_cap)
{
  return 3 * 3 * 8 * 64 * w_cap + 3 * 8 * u_cap + 2 * 64 * w_cap + 64 * 8 + 64 * 4 + 64 + ((64 * w_cap + 15) & ~15);
}

template <int MAXC, int MAXW, int UMODE>
__global__ __launch_bounds__(192) void k_assemble_elast_wg(int64_t n_slices, const SliceRec* __restrict__ recs,
                                                           unsigned long long* __restrict__ tickets, int u_cap,
                                                           int w_cap, bool per_block, const int32_t* __restrict__ perm,
                                                           const int64_t* __restrict__ pos_rb,
                                                           const uint32_t* __restrict__ pos_dl,
                                                           const uint8_t* __restrict__ strip,
                                                           const uint16_t* __restrict__ lidx,
                                                           const int32_t* __restrict__ snode,
                                                           const double* __restrict__ coords, double lambda, double mu,
                                                           double c0, double fx, double fy, double fz,
                                                           double* __restrict__ vals, double* __restrict__ rhs,
                                                           int rhs_add, const uint8_t* __restrict__ strip_u,
                                                           const SlotRec* __restrict__ uslots)
{
  const ElastK ek = elast_consts(lambda, mu, c0);
  // UMODE = 1 (uniform slices, as the scalar uniform instance): the slot bytes
  // come from the slice's common 32-B slot stream (scalar loads), each step's
  // coordinates from the lane's local-index stream (strip_u): no column-index
  // table in LDS, no dependent LDS read per step
  // UMODE = 3 (stencil): the same with the step bytes and shift/swap bits of
  // compiled-in signature 0 (the interior brick; rec_k0): accumulator offsets
  // are immediates, the shift/swap arms fixed at compile time
  constexpr bool ULOC = UMODE == 1 || UMODE == 3;
  extern __shared__ __align__(16) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int ci = __builtin_amdgcn_readfirstlane(tid >> 6);  // component row of this wave
  const int64_t acc_stride = 3 * 64 * (int64_t)w_cap;   // doubles per wave region
  double* const acc_all = reinterpret_cast<double*>(smem);
  double* const acc = acc_all + ci * acc_stride;  // [slot][k][lane]
  double* const cs = acc_all + 3 * acc_stride;    // SoA coordinates [3][u_cap]
  uint16_t* const li = reinterpret_cast<uint16_t*>(cs + 3 * (int64_t)u_cap);
  int64_t* const rbs = reinterpret_cast<int64_t*>(li + 64 * (int64_t)w_cap);
  int32_t* const fps = reinterpret_cast<int32_t*>(rbs + 64);
  unsigned long long* const claim = reinterpret_cast<unsigned long long*>(fps + 64);
  uint8_t* const bown = reinterpret_cast<uint8_t*>(claim + 8);  // block -> owning row lane
  const int xcd = (int)(blockIdx.x & 7);
  const int64_t r0 = n_slices * xcd / 8, r1 = n_slices * (xcd + 1) / 8;
  // workgroup claims: thread 0 takes a ticket, the workgroup reads it after a barrier
  auto issue = [&]() -> unsigned long long { return tid == 0 ? atomicAdd(tickets + 16 * xcd, 1ull) : 0ull; };
  auto uni = [&](unsigned long long t) -> int64_t {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)t);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(t >> 32));
    return r0 + (int64_t)(((uint64_t)hi << 32) | lo);
  };
  auto bcast = [&](unsigned long long t) -> int64_t {
    if (tid == 0) claim[0] = t;
    __syncthreads();
    const unsigned long long v = claim[0];
    __syncthreads();
    return uni(v);
  };
  int64_t p0 = bcast(issue());
  if (p0 >= r1) return;
  int64_t p1 = bcast(issue());
  int64_t p2 = bcast(issue());
  int64_t p3 = bcast(issue());
  SliceRec R0 = recs[p0];
  SliceRec R1 = recs[p1 < r1 ? p1 : p0];
  SliceRec R2 = recs[p2 < r1 ? p2 : p0];
  SlotRec S0{}, S1{}, S2{};
  if constexpr (UMODE == 1) {
    S0 = uslots[p0];
    S1 = uslots[p1 < r1 ? p1 : p0];
    S2 = uslots[p2 < r1 ? p2 : p0];
  }

  // staging share of a thread: nodes u = tid and tid + 192 (u_cap <= 256)
  auto load_nid = [&](const SliceRec& R, int32_t(&nid)[2]) {
    const int nu = (int)(R.meta & 0xFFFFu);
#pragma unroll
    for (int k = 0; k < 2; ++k) nid[k] = snode[(int64_t)R.snode_off + max(min(tid + 192 * k, nu - 1), 0)];
  };
  struct Pre {
    int32_t row;
    uint32_t dl;
    int64_t rb;
    u32x4 l0, l1;
    u32x4 ch[MAXC];
    u32x4 cu[MAXC];
    double x[2], y[2], z[2];
  };
  auto load_rows = [&](const SliceRec& R, Pre& p) {
    const int64_t q = (int64_t)R.sl * 64 + lane;
    p.row = perm[q];
    p.dl = pos_dl[q];
    p.rb = pos_rb[q];
    const int nc = (int)((R.meta >> 24) + 15) >> 4;
    if constexpr (ULOC) {
      const u32x4* su = reinterpret_cast<const u32x4*>(strip_u + (int64_t)R.strip_off * 1024) + lane;
#pragma unroll
      for (int c = 0; c < MAXC; ++c) p.cu[c] = su[(int64_t)max(min(c, nc - 1), 0) * 64];
    }
    else {
      if (ci == 0) {  // the column-index table (staged by wave 0)
        const int nq = 8 * (int)((R.meta >> 16) & 0xFFu);
        const u32x4* ls = reinterpret_cast<const u32x4*>(lidx + R.lidx_off);
        p.l0 = ls[max(min(lane, nq - 1), 0)];
        p.l1 = ls[max(min(lane + 64, nq - 1), 0)];
      }
      const u32x4* sp = reinterpret_cast<const u32x4*>(strip + (int64_t)R.strip_off * 1024) + lane;
#pragma unroll
      for (int c = 0; c < MAXC; ++c) p.ch[c] = sp[(int64_t)max(min(c, nc - 1), 0) * 64];
    }
  };
  auto gather = [&](const int32_t(&nid)[2], Pre& p) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      p.x[k] = coords[3 * (int64_t)nid[k]];
      p.y[k] = coords[3 * (int64_t)nid[k] + 1];
      p.z[k] = coords[3 * (int64_t)nid[k] + 2];
    }
  };
  Pre cur, nxt;
  int32_t nid1[2], nid2[2];
  {
    int32_t nid0[2];
    load_nid(R0, nid0);
    load_rows(R0, cur);
    gather(nid0, cur);
    load_nid(R1, nid1);
  }
  __builtin_amdgcn_s_waitcnt(0);
  // rotated-frame component arrays of this wave: (x_ci, x_ci+1, x_ci+2)
  const double* const ca = cs + (int64_t)u_cap * ci;
  const double* const cb = cs + (int64_t)u_cap * (ci == 2 ? 0 : ci + 1);
  const double* const cc = cs + (int64_t)u_cap * (ci == 0 ? 2 : ci - 1);
  for (;;) {
    const unsigned long long t4 = issue();  // read at the end of this iteration
    const SliceRec R3 = recs[p3 < r1 ? p3 : p0];
    SlotRec S3{};
    if constexpr (UMODE == 1) S3 = uslots[p3 < r1 ? p3 : p0];
    const int nsteps = (int)(R0.meta >> 24);
    const int W = (int)((R0.meta >> 16) & 0xFFu);
    const int nu = (int)(R0.meta & 0xFFFFu);
    // ---- stage: coordinates (SoA), column indices, zero accumulators
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int u = tid + 192 * k;
      if (u < nu) {
        cs[u] = cur.x[k];
        cs[u_cap + u] = cur.y[k];
        cs[2 * u_cap + u] = cur.z[k];
      }
    }
    if (!ULOC && ci == 0) {
      const int nq = 8 * W;
      u32x4* dst = reinterpret_cast<u32x4*>(li);
      dst[max(min(lane, nq - 1), 0)] = cur.l0;
      dst[max(min(lane + 64, nq - 1), 0)] = cur.l1;
    }
    if constexpr (UMODE != 3) {  // the stencil instance stores every slot's first contribution
      double2* a2 = reinterpret_cast<double2*>(acc);
      for (int q = lane; q < 96 * W; q += 64) a2[q] = make_double2(0.0, 0.0);
    }
    __syncthreads();
    load_rows(R1, nxt);
    gather(nid1, nxt);
    load_nid(R2, nid2);

    const int32_t row = cur.row;
    const bool active = row >= 0;
    const int64_t rb = cur.rb;
    const int len = (int)((cur.dl >> 8) & 0xFFu);
    const uint32_t dslot = cur.dl & 0xFFu;
    const uint16_t* lrow = li + lane;
    auto coord = [&](int u) { return V3{ ca[u], cb[u], cc[u] }; };
    const V3 xi = coord(ULOC ? (int)(cur.dl >> 16) : (int)lrow[dslot * 64]);
    double macc = 0.0;
    V3 eP{ 0.0, 0.0, 0.0 }, eQ{ 0.0, 0.0, 0.0 }, eR{ 0.0, 0.0, 0.0 };
    V3 cP{ 0.0, 0.0, 0.0 }, cN{ 0.0, 0.0, 0.0 };
    double* const acc_lane = acc + lane;
    double* aP = acc_lane + 192 * dslot;
    double* aQ = aP;
    double* aR = aP;
    // Register window: the partial sums of the three window nodes' entries
    // stay in registers (gP, gQ, gR) while the node is in the window; a node
    // leaving it (one per step: P on a shift, Q on a swap) is flushed into its
    // LDS accumulators.  3 ds_add_f64 per step instead of 9; the entry of a
    // (row, column) is summed per window visit first, then over the visits
    // (fixed order: still bitwise reproducible, the same in both instances).
    V3 gP{ 0.0, 0.0, 0.0 }, gQ{ 0.0, 0.0, 0.0 }, gR{ 0.0, 0.0, 0.0 };
    auto lidx_of = [&](uint32_t byte) { return (int)lrow[(byte & 63u) * 64]; };
    auto sel = [](bool c, V3 a, V3 b) { return V3{ c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z }; };
    auto keep = [](uint64_t m, double x) { return __longlong_as_double((long long)(m & (uint64_t)__double_as_longlong(x))); };
    auto byte_at = [&](int j) -> uint32_t {
      if constexpr (ULOC) {  // scalar: the slice's common slot stream
        return (S0.w[(j >> 2) & 7] >> (8 * (j & 3))) & 0xFFu;
      }
      else {
        const u32x4 w = cur.ch[j >> 4];
        const int q = (j >> 2) & 3;
        const uint32_t wq = q == 0 ? w.x : (q == 1 ? w.y : (q == 2 ? w.z : w.w));
        return (wq >> (8 * (j & 3))) & 0xFFu;
      }
    };
    auto uloc_at = [&](int j) -> int {  // local node index of step j (ULOC)
      const u32x4 w = cur.cu[j >> 4];
      const int q = (j >> 2) & 3;
      const uint32_t wq = q == 0 ? w.x : (q == 1 ? w.y : (q == 2 ? w.z : w.w));
      return (int)((wq >> (8 * (j & 3))) & 0xFFu);
    };
    constexpr int NSTEP = 16 * MAXC;
    if constexpr (ULOC) {
      auto ustep = [&](auto swap_c, auto first_c, uint32_t byte, V3 xd) {
        constexpr bool SWAP = decltype(swap_c)::value;
        constexpr bool FIRST = decltype(first_c)::value;
        double* const aD = acc_lane + 192 * (byte & 63u);
        const V3 eD = sub(xd, xi);
        V3 cRn;
        if constexpr (SWAP) {
          cRn = cN;
          if constexpr (FIRST) store3(aQ, gQ);
          else flush3(aQ, gQ);
        }
        else {
          cRn = cP;
          eP = eQ;
          if constexpr (FIRST) store3(aP, gP);
          else flush3(aP, gP);
          aP = aQ;
          gP = gQ;
        }
        eQ = eR;
        aQ = aR;
        gQ = gR;
        eR = eD;
        aR = aD;
        cP = cross(eQ, eR);
        cN = cross(eP, eR);
        const V3 m = V3{ cP.x - cN.x + cRn.x, cP.y - cN.y + cRn.y, cP.z - cN.z + cRn.z };
        const double meas = fabs(dot(eP, cP));
        const double s = -recip1(UMODE == 3 ? meas : fmax(meas, 1e-300));
        const double mass = meas * ek.m120;
        macc += meas;
        const ElastPre e = elast_pre(m, s, ek);
        gP = elast_acc(gP, e, cP, mass);
        gQ = elast_acc(gQ, e, V3{ -cN.x, -cN.y, -cN.z }, mass);
        gR = elast_first(e, cRn, mass);
      };
      // bytes(j): step j's byte, swp(j): step j is a swap (scalar, or constants)
      auto run = [&](auto bytes, auto swp, auto fst) {
        {
          const uint32_t b0 = bytes(0), b1 = bytes(1);
          eQ = sub(coord(uloc_at(0)), xi);
          eR = sub(coord(uloc_at(1)), xi);
          aQ = acc_lane + 192 * (b0 & 63u);
          aR = acc_lane + 192 * (b1 & 63u);
          cP = cross(eQ, eR);
        }
        V3 xc = coord(uloc_at(2));
#pragma unroll
        for (int j = 2; j < NSTEP; ++j) {
          if ((j & 1) == 0 && j >= nsteps) break;
          const V3 xn = j + 1 < NSTEP ? coord(uloc_at(j + 1 < NSTEP ? j + 1 : j)) : xc;
          if (fst(j)) {
            if (swp(j)) ustep(std::true_type{}, std::true_type{}, bytes(j), xc);
            else ustep(std::false_type{}, std::true_type{}, bytes(j), xc);
          }
          else {
            if (__builtin_expect(swp(j), 0)) ustep(std::true_type{}, std::false_type{}, bytes(j), xc);
            else ustep(std::false_type{}, std::false_type{}, bytes(j), xc);
          }
          xc = xn;
        }
      };
      if constexpr (UMODE == 1) {
        const uint64_t pat = R0.pat;
        run(byte_at, [&](int j) { return ((pat >> j) & 1u) != 0; }, [](int) { return false; });
      }
      else {
        // the list holds the slices of signature 0 (the interior brick) only (one
        // unrolled body: a second one in the same kernel spilled to scratch)
        constexpr const StencilSig& S = *kStencilSigPtrs[0];
        run([](int j) -> uint32_t { return j < S.nsteps ? S.slot[j] : (uint32_t)(0xC0 | S.dslot); },
            [](int j) { return ((S.pat >> j) & 1u) != 0; },
            [](int j) { return j < S.nsteps && kStencilWin<S>.first[j]; });
      }
    }
    else {
      auto step = [&](uint32_t byte, V3 xd) {
        const bool swap = (byte & 0xC0u) == 0x40u;
        const uint64_t em = (uint64_t)0 - (uint64_t)(byte < 0x80u);
        double* const aD = acc_lane + 192 * (byte & 63u);
        const V3 eD = sub(xd, xi);
        const V3 cRn = sel(swap, cN, cP);
        eP = sel(swap, eP, eQ);
        flush3(swap ? aQ : aP, sel(swap, gQ, gP));
        gP = sel(swap, gP, gQ);
        aP = swap ? aP : aQ;
        eQ = eR;
        aQ = aR;
        gQ = gR;
        eR = eD;
        aR = aD;
        cP = cross(eQ, eR);
        cN = cross(eP, eR);
        const V3 m = V3{ cP.x - cN.x + cRn.x, cP.y - cN.y + cRn.y, cP.z - cN.z + cRn.z };
        const double meas = fabs(dot(eP, cP));
        const double s = keep(em, -recip1(meas));
        const double mass = keep(em, meas * ek.m120);
        macc += keep(em, meas);
        const ElastPre e = elast_pre(m, s, ek);
        gP = elast_acc(gP, e, cP, mass);
        gQ = elast_acc(gQ, e, V3{ -cN.x, -cN.y, -cN.z }, mass);
        gR = elast_first(e, cRn, mass);
      };
      int u1 = lidx_of(byte_at(0));
      V3 xc = coord(u1);
      u1 = lidx_of(byte_at(1));
#pragma unroll
      for (int j = 0; j < NSTEP; ++j) {
        if ((j & 3) == 0 && j >= nsteps) break;
        const int u2 = j + 2 < NSTEP ? lidx_of(byte_at(j + 2)) : 0;
        const V3 xn = j + 1 < NSTEP ? coord(u1) : xc;
        step(byte_at(j), xc);
        xc = xn;
        u1 = u2;
      }
    }
    if constexpr (UMODE == 3) {
      constexpr const StencilSig& S = *kStencilSigPtrs[0];
      if (kStencilWin<S>.fin[0]) store3(aP, gP);
      else flush3(aP, gP);
      if (kStencilWin<S>.fin[1]) store3(aQ, gQ);
      else flush3(aQ, gQ);
      if (kStencilWin<S>.fin[2]) store3(aR, gR);
      else flush3(aR, gR);
    }
    else {
      flush3(aP, gP);
      flush3(aQ, gQ);
      flush3(aR, gR);
    }
    if (rhs && active) {
      const double rv = (ci == 0 ? fx : (ci == 1 ? fy : fz)) * macc * (1.0 / 24.0);
      st_out(&rhs[3 * (int64_t)row + ci], rhs_add ? rhs[3 * (int64_t)row + ci] + rv : rv);
    }
    wave_sync_lds();

    // ---- diagonal block row, then the slice's complete blocks through one flat image
    int fp = len;  // block prefix over the lanes (the same in the three waves)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(fp, o);
      if (lane >= o) fp += t;
    }
    const int total = __shfl(fp, 63);  // blocks of the slice
    fp -= len;
    double rv[3 * MAXW];
    double sum[3] = { 0.0, 0.0, 0.0 };
    if constexpr (UMODE == 3) {
      // the signature's slots at constant offsets; the diagonal slot is skipped
      // (the other instances add its zeroed accumulator: +0, the same sums)
      constexpr int WS0 = kStencilSigPtrs[0]->w, DS0 = kStencilSigPtrs[0]->dslot;
#pragma unroll
      for (int t = 0; t < WS0; ++t)
        if (t != DS0)
#pragma unroll
          for (int k = 0; k < 3; ++k) rv[3 * t + k] = acc_lane[192 * t + 64 * k];
#pragma unroll
      for (int t = 0; t < WS0; ++t)
        if (t != DS0)
#pragma unroll
          for (int k = 0; k < 3; ++k) sum[k] += rv[3 * t + k];
    }
    else {
      if (active) {
        acc_lane[192 * dslot] = 0.0;
        acc_lane[192 * dslot + 64] = 0.0;
        acc_lane[192 * dslot + 128] = 0.0;
      }
#pragma unroll
      for (int t = 0; t < MAXW; ++t)
#pragma unroll
        for (int k = 0; k < 3; ++k) rv[3 * t + k] = acc_lane[192 * min(t, W - 1) + 64 * k];
#pragma unroll
      for (int t = 0; t < MAXW; ++t)
        if (t < W)
#pragma unroll
          for (int k = 0; k < 3; ++k) sum[k] += rv[3 * t + k];
    }
    // stencil instance, full slice (64 rows of the signature's length WS): row L's
    // values are flat positions [9 WS L, 9 WS (L + 1)) -- a division by a
    // constant instead of the owner / prefix tables
    constexpr int WS = UMODE == 3 ? kStencilSigPtrs[0]->w : 0;
    const bool full = UMODE == 3 && total == 64 * WS;
    if (ci == 0) {
      rbs[lane] = active ? rb : 0;
      if (!full) {
        fps[lane] = fp;
        for (int t = 0; t < len; ++t) bown[fp + t] = (uint8_t)lane;
      }
    }
    __syncthreads();  // every wave's accumulator reads before the flat image overwrites them
    double* const flat = acc_all;
    // value (t, k) of the rotated frame = block column j = (ci + k) % 3; the
    // block (row, t) holds 9 values: per block [i][j] at 9 t + 3 i + j, per
    // row (CSR order) at 3 len i + 3 t + j
    if (UMODE == 3 && full) {
      // every row: the signature's length and diagonal slot, prefix 9 WS lane
      constexpr int DS = UMODE == 3 ? kStencilSigPtrs[0]->dslot : 0;
      double* const fr = flat + 9 * WS * lane + (per_block ? 3 * ci : 3 * WS * ci);
#pragma unroll
      for (int t = 0; t < WS; ++t)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int j = k + ci < 3 ? k + ci : k + ci - 3;
          const double v = t == DS ? add_nc(-sum[k], k == 0 ? c0 * macc * (1.0 / 24.0) : 0.0) : rv[3 * t + k];
          fr[(per_block ? 9 * t : 3 * t) + j] = v;
        }
    }
    else if (active) {
#pragma unroll
      for (int t = 0; t < MAXW; ++t)
        if (t < len) {
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            const int j = k + ci < 3 ? k + ci : k + ci - 3;
            const double v = t == (int)dslot ? add_nc(-sum[k], k == 0 ? c0 * macc * (1.0 / 24.0) : 0.0) : rv[3 * t + k];
            flat[9 * fp + (per_block ? 9 * t + 3 * ci + j : 3 * len * ci + 3 * t + j)] = v;
          }
        }
    }
    if (tid == 0) claim[0] = t4;
    __syncthreads();
    const int64_t pn = uni(claim[0]);
    // store: flat position P is value P - 9 fps[L] of row lane L = bown[P / 9]
    if (UMODE == 3 && full) {
      constexpr int B = 9 * (WS > 0 ? WS : 1);
      // brick x-runs: lanes 4q..4q+3 hold consecutive rows of the same length,
      // so their 4B values are one contiguous range at 9 rb(4q) (both layouts:
      // a node row's 9 len values are contiguous in either) -- the run's base is
      // a wave-uniform scalar, each thread's offsets are constants: no
      // per-value owner division, no dependent LDS read, no 64-bit address math
      const int64_t rb_run = __shfl(rb, lane & ~3);
      if (__all(rb == rb_run + (int64_t)WS * (lane & 3))) {
        constexpr int RUN = 4 * B;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)rb, 4 * r);
          const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)rb >> 32), 4 * r);
          double* const dst = vals + 9 * (int64_t)(((uint64_t)hi << 32) | lo);
          const double* const src = flat + RUN * r;
#if AFEM_WG_ST16
          // 16 B per thread (values 2 o', 2 o' + 1; the run start is 8-B aligned:
          // unaligned 16-B stores), threads past the run repeat its last pair
          // (same addresses, same values): 2 stores per thread and run, not 3
          typedef double d2u __attribute__((ext_vector_type(2), aligned(8)));
          static_assert(RUN % 2 == 0, "pairs");
#pragma unroll
          for (int i = 0; i < (RUN / 2 + 191) / 192; ++i) {
            const int o = min(2 * (tid + 192 * i), RUN - 2);
#if AFEM_WG_NT
            __builtin_nontemporal_store(d2u{ src[o], src[o + 1] }, reinterpret_cast<d2u*>(dst + o));
#else
            st_out(reinterpret_cast<d2u*>(dst + o), d2u{ src[o], src[o + 1] });
#endif
          }
#else
#pragma unroll
          for (int i = 0; i < (RUN + 191) / 192; ++i) {
            // threads past the run repeat its last value (same address and
            // value): no exec-mask branch between the image reads
            const int o = min(tid + 192 * i, RUN - 1);
            st_out(&dst[o], src[o]);
          }
#endif
        }
      }
      else {
        for (int P = tid; P < 64 * B; P += 192) {
          const int L = P / B;
          st_out(&vals[9 * rbs[L] + (P - L * B)], flat[P]);
        }
      }
    }
    else {
      for (int P = tid; P < 9 * total; P += 192) {
        const int L = bown[P / 9];
        st_out(&vals[9 * rbs[L] + (P - 9 * fps[L])], flat[P]);
      }
    }
    __syncthreads();
    if (p1 >= r1) break;
    p0 = p1;
    p1 = p2;
    p2 = p3;
    p3 = pn;
    R0 = R1;
    R1 = R2;
    R2 = R3;
    if constexpr (UMODE == 1) {
      S0 = S1;
      S1 = S2;
      S2 = S3;
    }
    cur = nxt;
#pragma unroll
    for (int k = 0; k < 2; ++k) nid1[k] = nid2[k];
  }
}

// ---------------------------------------------------------------- block-3 elasticity (TETRA4), row strips
// K_rb^{ij} = [lambda c_r,i c_b,j + mu (c_r,j c_b,i + delta_ij c_r.c_b)] / (6|det|)
// (+ c0 |det|/120 delta_ij, the consistent mass V/20 (1 + delta_rb) for b != r):
// the 3D form of computeElementMatrixTRIA3Base (modules/elasticity/FemModule.h:112-140),
// restated in oracle/oracle.c orc_element_elasticity_tet4.  One wave per
// (slice, component row i): it walks the slice's row strips exactly like the
// scalar kernel and accumulates the three entries (i, j=0..2) of every
// block of its 64 rows in LDS [slot][j][lane].  Diagonal blocks: rigid
// translations are in the nullspace, so K_rr = -sum_{b != r} K_rb; the mass
// part (row sum V/4, diagonal V/10) is restored from the row's measure sum.
// Body force f (vectorial constant source, femutils/ArcaneFemFunctionsGpu.h:514-586):
// rhs[3r+i] = f_i |K|/4, fused.
template <int MAXW>
__global__ __launch_bounds__(64) void k_assemble_elast_tet(int u_cap, int w_cap, bool per_block,
                                                           const int32_t* __restrict__ perm,
                                                           const int64_t* __restrict__ row_ptr,
                                                           const uint8_t* __restrict__ strip,
                                                           const int64_t* __restrict__ strip_ptr,
                                                           const int32_t* __restrict__ strip_n,
                                                           const uint8_t* __restrict__ dslots,
                                                           const int32_t* __restrict__ slice_w,
                                                           const int64_t* __restrict__ lidx_ptr,
                                                           const uint16_t* __restrict__ lidx,
                                                           const int64_t* __restrict__ snode_ptr,
                                                           const int32_t* __restrict__ snode,
                                                           const double* __restrict__ coords, double lambda, double mu,
                                                           double c0, double fx, double fy, double fz,
                                                           double* __restrict__ vals, double* __restrict__ rhs, int rhs_add)
{
  extern __shared__ __align__(16) unsigned char smem[];
  double* acc = reinterpret_cast<double*>(smem);  // [slot][j][lane]
  double* cxyz = reinterpret_cast<double*>(smem + 3 * 8 * 64 * (int64_t)w_cap);
  uint16_t* li = reinterpret_cast<uint16_t*>(reinterpret_cast<unsigned char*>(cxyz) +
                                             ((24 * (int64_t)u_cap + 15) & ~int64_t(15)));
  const int lane = threadIdx.x;
  const int64_t sl = blockIdx.x / 3;
  const int ci = (int)(blockIdx.x % 3);  // component row of this wave (uniform)
  const int32_t row = perm[sl * 64 + lane];
  const bool active = row >= 0;
  const int64_t rb = active ? row_ptr[row] : 0;
  const int len = active ? (int)(row_ptr[row + 1] - rb) : 0;
  const V3 xi = ld3(coords, active ? row : 0);
  const uint32_t dslot = dslots[sl * 64 + lane];
  const int W = slice_w[sl];
  const int nsteps = strip_n[sl];
  // stage coordinates (AoS), column-index table, zero accumulators
  {
    const int64_t u0 = snode_ptr[sl];
    const int nu = (int)(snode_ptr[sl + 1] - u0);
    for (int u = lane; u < nu; u += 64) {
      const int64_t n = snode[u0 + u];
      cxyz[3 * u] = coords[3 * n];
      cxyz[3 * u + 1] = coords[3 * n + 1];
      cxyz[3 * u + 2] = coords[3 * n + 2];
    }
    const int nq = 8 * W;
    const u32x4* ls = reinterpret_cast<const u32x4*>(lidx + lidx_ptr[sl]);
    u32x4* dst = reinterpret_cast<u32x4*>(li);
    for (int q = lane; q < nq; q += 64) dst[q] = ls[q];
    double2* a2 = reinterpret_cast<double2*>(acc);
    for (int q = lane; q < 96 * W; q += 64) a2[q] = make_double2(0.0, 0.0);
  }
  wave_sync_lds();

  const double* comp_sel = nullptr;
  (void)comp_sel;
  double macc = 0.0;
  V3 eP{ 0.0, 0.0, 0.0 }, eQ{ 0.0, 0.0, 0.0 }, eR{ 0.0, 0.0, 0.0 };
  V3 cP{ 0.0, 0.0, 0.0 }, cN{ 0.0, 0.0, 0.0 };
  double* const acc_lane = acc + lane;
  double* aP = acc_lane + 192 * dslot;
  double* aQ = aP;
  double* aR = aP;
  const uint16_t* lrow = li + lane;
  const u32x4* sp = reinterpret_cast<const u32x4*>(strip + strip_ptr[sl]) + lane;
  auto comp = [ci](V3 v) { return ci == 0 ? v.x : (ci == 1 ? v.y : v.z); };
  auto sel = [](bool c, V3 a, V3 b) { return V3{ c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z }; };
  auto keep = [](uint64_t m, double x) { return __longlong_as_double((long long)(m & (uint64_t)__double_as_longlong(x))); };
  auto block = [&](double* a, V3 m, V3 cb, double s, double mass) {
    // entries (ci, j) of K_rb with c_r = -m (sign folded into s < 0)
    const double t = dot(m, cb);
    const double A = lambda * comp(m), B = mu * comp(cb);
    double v0 = (A * cb.x + B * m.x) * s, v1 = (A * cb.y + B * m.y) * s, v2 = (A * cb.z + B * m.z) * s;
    const double dg = mu * t * s + mass;
    if (ci == 0) v0 += dg;
    else if (ci == 1) v1 += dg;
    else v2 += dg;
    atomicAdd(a, v0);
    atomicAdd(a + 64, v1);
    atomicAdd(a + 128, v2);
  };
  for (int c = 0; 16 * c < nsteps; ++c) {
    const u32x4 w = sp[(int64_t)c * 64];
    const uint32_t wv[4] = { w.x, w.y, w.z, w.w };
    for (int j = 0; j < 16; ++j) {
      const uint32_t byte = (wv[j >> 2] >> (8 * (j & 3))) & 0xFFu;
      const bool swap = (byte & 0xC0u) == 0x40u;
      const uint64_t em = (uint64_t)0 - (uint64_t)(byte < 0x80u);
      double* const aD = acc_lane + 192 * (byte & 63u);
      const double* q = cxyz + 3 * (int)lrow[(byte & 63u) * 64];
      const V3 eD = sub(V3{ q[0], q[1], q[2] }, xi);
      const V3 cRn = sel(swap, cN, cP);
      eP = sel(swap, eP, eQ);
      aP = swap ? aP : aQ;
      eQ = eR;
      aQ = aR;
      eR = eD;
      aR = aD;
      cP = cross(eQ, eR);
      cN = cross(eP, eR);
      const V3 m = V3{ cP.x - cN.x + cRn.x, cP.y - cN.y + cRn.y, cP.z - cN.z + cRn.z };
      const double meas = fabs(dot(eP, cP));
      const double s = keep(em, -recip1(6.0 * meas));
      const double mass = keep(em, c0 * meas * (1.0 / 120.0));
      macc += keep(em, meas);
      block(aP, m, cP, s, mass);
      block(aQ, m, V3{ -cN.x, -cN.y, -cN.z }, s, mass);
      block(aR, m, cRn, s, mass);
    }
  }
  if (rhs && active) {
    const double rv = (ci == 0 ? fx : (ci == 1 ? fy : fz)) * macc * (1.0 / 24.0);
    st_out(&rhs[3 * (int64_t)row + ci], rhs_add ? rhs[3 * (int64_t)row + ci] + rv : rv);
  }
  wave_sync_lds();
  // diagonal block row ci, then the row's 3*len values
  if (active) {
    double sum[3] = { 0.0, 0.0, 0.0 };
    for (int t = 0; t < len; ++t)
      if (t != (int)dslot)
        for (int jj = 0; jj < 3; ++jj) sum[jj] += acc_lane[192 * t + 64 * jj];
    for (int jj = 0; jj < 3; ++jj)
      acc_lane[192 * dslot + 64 * jj] = add_nc(-sum[jj], jj == ci ? c0 * macc * (1.0 / 24.0) : 0.0);
    for (int t = 0; t < len; ++t)
      for (int jj = 0; jj < 3; ++jj)
        st_out(&vals[per_block ? (rb + t) * 9 + 3 * ci + jj : rb * 9 + (int64_t)ci * 3 * len + 3 * t + jj],
          acc_lane[192 * t + 64 * jj]);
  }
}

// Global-memory variant for rows too long for the LDS tile: coordinates
// gathered through the columns, accumulation in place (lane-owned rows).
template <int NV>
__global__ __launch_bounds__(64) void k_assemble_p1_global(const int32_t* __restrict__ perm,
                                                           const int64_t* __restrict__ row_ptr,
                                                           const int32_t* __restrict__ cols,
                                                           const uint32_t* __restrict__ inc,
                                                           const int64_t* __restrict__ slice_ptr,
                                                           const int32_t* __restrict__ slice_k,
                                                           const double* __restrict__ coords, double s_coef,
                                                           double f_meas, double* __restrict__ vals,
                                                           double* __restrict__ rhs, int rhs_add)
{
  const int lane = threadIdx.x;
  const int64_t sl = blockIdx.x;
  const int32_t row = perm[sl * 64 + lane];
  if (row < 0) return;
  const int64_t rb = row_ptr[row];
  const int len = (int)(row_ptr[row + 1] - rb);
  const int32_t* crow = cols + rb;
  double* arow = vals + rb;
  for (int t = 0; t < len; ++t) arow[t] = 0.0;
  const V3 xi = ld3(coords, row);
  const uint32_t* ip = inc + slice_ptr[sl] + lane * 4;
  const int kmax = slice_k[sl];
  double dacc = 0.0, macc = 0.0;
  uint32_t dslot = 0xFFu;
  for (int k = 0; k < kmax; ++k) {
    const uint32_t e = ip[(int64_t)(k >> 2) * 256 + (k & 3)];
    if (e == kPad) break;
    dslot = e >> 24;
    const V3 xa = ld3(coords, crow[e & 0xFFu]), xb = ld3(coords, crow[(e >> 8) & 0xFFu]);
    double k0, k1, k2, k3 = 0.0, meas;
    if (NV == 4)
      meas = tet_row(xi, xa, xb, ld3(coords, crow[(e >> 16) & 0xFFu]), s_coef, k0, k1, k2, k3);
    else
      meas = tri_row(xi, xa, xb, s_coef, k0, k1, k2);
    dacc += k0;
    macc += meas;
    arow[e & 0xFFu] += k1;
    arow[(e >> 8) & 0xFFu] += k2;
    if (NV == 4) arow[(e >> 16) & 0xFFu] += k3;
  }
  if (dslot != 0xFFu) arow[dslot] = dacc;
  if (rhs) rhs[row] = rhs_add ? rhs[row] + f_meas * macc : f_meas * macc;
}

// Block-3 global-memory variant for meshes without row strips (a node with
// more than 64 incident cells, rows of more than 64 blocks): one wave per
// (slice, component row ci), lane-owned rows, the incidence table gives the
// row-slots of each incident cell's other nodes, coordinates gathered through
// the columns, entries accumulated in place (each value has one writer).
// Same element matrix as the strip kernels (orc_element_elasticity_tet4):
// K_rb^{ij} = [lambda c_r,i c_b,j + mu (c_r,j c_b,i + d_ij c_r.c_b)] / (6|det|)
// + c0 |det|/120 (1 + d_rb) d_ij, c the cofactors (gradients x det).
__global__ __launch_bounds__(64) void k_assemble_elast_tet_global(
    bool per_block, const int32_t* __restrict__ perm, const int64_t* __restrict__ row_ptr,
    const int32_t* __restrict__ cols, const uint32_t* __restrict__ inc, const int64_t* __restrict__ slice_ptr,
    const int32_t* __restrict__ slice_k, const double* __restrict__ coords, double lambda, double mu, double c0,
    double fx, double fy, double fz, double* __restrict__ vals, double* __restrict__ rhs, int rhs_add)
{
  const int lane = threadIdx.x;
  const int64_t sl = blockIdx.x / 3;
  const int ci = (int)(blockIdx.x % 3);
  const int32_t row = perm[sl * 64 + lane];
  if (row < 0) return;
  const int64_t rb = row_ptr[row];
  const int len = (int)(row_ptr[row + 1] - rb);
  auto vidx = [&](int t, int j) -> int64_t {
    return per_block ? (rb + t) * 9 + 3 * ci + j : rb * 9 + (int64_t)ci * 3 * len + 3 * t + j;
  };
  for (int t = 0; t < len; ++t)
    for (int j = 0; j < 3; ++j) vals[vidx(t, j)] = 0.0;
  const int32_t* crow = cols + rb;
  const V3 xi = ld3(coords, row);
  const uint32_t* ip = inc + slice_ptr[sl] + lane * 4;
  const int kmax = slice_k[sl];
  auto comp = [](V3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); };
  double macc = 0.0;
  for (int k = 0; k < kmax; ++k) {
    const uint32_t e = ip[(int64_t)(k >> 2) * 256 + (k & 3)];
    if (e == kPad) break;
    const int slot[4] = { (int)(e >> 24), (int)(e & 0xFFu), (int)((e >> 8) & 0xFFu), (int)((e >> 16) & 0xFFu) };
    const V3 e1 = sub(ld3(coords, crow[slot[1]]), xi), e2 = sub(ld3(coords, crow[slot[2]]), xi),
             e3 = sub(ld3(coords, crow[slot[3]]), xi);
    const V3 c1 = cross(e2, e3), c2 = cross(e3, e1), c3 = cross(e1, e2);
    const V3 cr = V3{ -(c1.x + c2.x + c3.x), -(c1.y + c2.y + c3.y), -(c1.z + c2.z + c3.z) };
    const double meas = fabs(dot(e1, c1));
    const double s = 1.0 / (6.0 * meas);
    const double mass = c0 * meas * (1.0 / 120.0);
    macc += meas;
    const V3 cb[4] = { cr, c1, c2, c3 };
    for (int b = 0; b < 4; ++b) {
      const double t = dot(cr, cb[b]);
      for (int j = 0; j < 3; ++j) {
        double v = (lambda * comp(cr, ci) * comp(cb[b], j) + mu * (comp(cr, j) * comp(cb[b], ci) + (ci == j ? t : 0.0))) * s;
        if (ci == j) v += b == 0 ? 2.0 * mass : mass;
        vals[vidx(slot[b], j)] += v;
      }
    }
  }
  if (rhs) {
    const double rv = (ci == 0 ? fx : (ci == 1 ? fy : fz)) * macc * (1.0 / 24.0);
    rhs[3 * (int64_t)row + ci] = rhs_add ? rhs[3 * (int64_t)row + ci] + rv : rv;
  }
}

// ---------------------------------------------------------------- block-2 elasticity (TRIA3)
// Element matrix of modules/elasticity/FemModule.h:112-140 restricted to the
// two rows of the row node (row node first; the 6x6 matrix is covariant
// under node permutations).  Values either ordered per block
// (blk*4 + i*2 + j) or per scalar row (CSR order, Hypre layout):
// start*4 + i*2*nnz_row + 2*slot + j.
__device__ __forceinline__ int64_t bidx2(bool per_block, int64_t rb4, int64_t nnz_row, int slot, int i, int j)
{
  return per_block ? rb4 + (int64_t)slot * 4 + i * 2 + j : rb4 + (int64_t)i * 2 * nnz_row + 2 * slot + j;
}

template <bool LDS>
__global__ __launch_bounds__(64) void k_assemble_elast_tri(int u_cap, int w_cap, int run, bool per_block,
                                                           const int32_t* __restrict__ perm,
                                                           const int64_t* __restrict__ row_ptr,
                                                           const int32_t* __restrict__ cols,
                                                           const uint32_t* __restrict__ inc,
                                                           const int64_t* __restrict__ slice_ptr,
                                                           const int32_t* __restrict__ slice_k,
                                                           const int32_t* __restrict__ slice_w,
                                                           const int64_t* __restrict__ lidx_ptr,
                                                           const uint16_t* __restrict__ lidx,
                                                           const int64_t* __restrict__ snode_ptr,
                                                           const int32_t* __restrict__ snode,
                                                           const double* __restrict__ coords, double lambda,
                                                           double mu2, double* __restrict__ vals)
{
  extern __shared__ __align__(16) unsigned char smem[];
  Tile<2, 4, 0> tile(smem, u_cap, w_cap);
  const int lane = threadIdx.x;
  const int64_t sl = xcd_swizzle(blockIdx.x, gridDim.x);
  const int32_t row = perm[sl * 64 + lane];
  const bool active = row >= 0;
  const int64_t rb = active ? row_ptr[row] : 0;
  const int len = active ? (int)(row_ptr[row + 1] - rb) : 0;
  const V3 x0 = ld3(coords, active ? row : 0);
  const uint32_t* ip = inc + slice_ptr[sl] + lane * 4;
  const int kmax = active ? slice_k[sl] : 0;
  if (LDS) {
    const int64_t u0 = snode_ptr[sl];
    tile.stage(lane, (int)(snode_ptr[sl + 1] - u0), snode + u0, coords, slice_w[sl], lidx + lidx_ptr[sl]);
  }
  else {
    for (int t = 0; t < 4 * len; ++t) vals[4 * rb + t] = 0.0;
  }
  const int32_t* crow = cols + rb;
  // accumulator of (slot, i, j): LDS tile, or the value array itself
  auto add = [&](int slot, int i, int j, double v) {
    if (LDS)
      atomicAdd(tile.at(lane, slot, 2 * i + j), v);
    else
      vals[bidx2(per_block, 4 * rb, len, slot, i, j)] += v;
  };
  auto put = [&](int slot, int i, int j, double v) {
    if (LDS)
      *tile.at(lane, slot, 2 * i + j) = v;
    else
      vals[bidx2(per_block, 4 * rb, len, slot, i, j)] = v;
  };
  if (active) {
    double d00 = 0, d01 = 0, d10 = 0, d11 = 0;
    uint32_t dslot = 0xFFu;
    for (int k = 0; k < kmax; ++k) {
      const uint32_t e = ip[(int64_t)(k >> 2) * 256 + (k & 3)];
      if (e == kPad) break;
      const int s[2] = { (int)(e & 0xFFu), (int)((e >> 8) & 0xFFu) };
      dslot = e >> 24;
      const V3 x1 = LDS ? tile.node(lane, s[0]) : ld3(coords, crow[s[0]]);
      const V3 x2 = LDS ? tile.node(lane, s[1]) : ld3(coords, crow[s[1]]);
      // 2A * grad N: dPhi0 = (y1-y2, x2-x1), dPhi1 = (y2-y0, x0-x2), dPhi2 = (y0-y1, x1-x0)
      const double px[3] = { x1.y - x2.y, x2.y - x0.y, x0.y - x1.y };
      const double py[3] = { x2.x - x1.x, x0.x - x2.x, x1.x - x0.x };
      const double e1x = x1.x - x0.x, e1y = x1.y - x0.y, e2x = x2.x - x0.x, e2y = x2.y - x0.y;
      const double area = fabs(e1x * e2y - e2x * e1y) / 2.0;
      const double sc = 1.0 / (4.0 * area);
      // row dof i of node 0, column dof j of node b:
      //  lam(i,j)  = (bx_i + by_i)(bx_j + by_j) over the interleaved B rows
      //  shr(i,j)  = bx_i bx_j + by_i by_j + 0.5 bs_i bs_j
      // with for dof (node a, comp 0): bx = px[a], by = 0, bs = py[a]
      //      for dof (node a, comp 1): bx = 0, by = py[a], bs = px[a]
      for (int nb = 0; nb < 3; ++nb) {
        const double K00 = (lambda * (px[0] * px[nb])) * sc + (mu2 * (px[0] * px[nb] + 0.5 * py[0] * py[nb])) * sc;
        const double K01 = (lambda * (px[0] * py[nb])) * sc + (mu2 * (0.5 * py[0] * px[nb])) * sc;
        const double K10 = (lambda * (py[0] * px[nb])) * sc + (mu2 * (0.5 * px[0] * py[nb])) * sc;
        const double K11 = (lambda * (py[0] * py[nb])) * sc + (mu2 * (py[0] * py[nb] + 0.5 * px[0] * px[nb])) * sc;
        if (nb == 0) {
          d00 += K00;
          d01 += K01;
          d10 += K10;
          d11 += K11;
        }
        else {
          const int sl2 = s[nb - 1];
          add(sl2, 0, 0, K00);
          add(sl2, 0, 1, K01);
          add(sl2, 1, 0, K10);
          add(sl2, 1, 1, K11);
        }
      }
    }
    if (dslot != 0xFFu) {
      put((int)dslot, 0, 0, d00);
      put((int)dslot, 0, 1, d01);
      put((int)dslot, 1, 0, d10);
      put((int)dslot, 1, 1, d11);
    }
  }
  if (LDS) write_back<4>(tile, lane, run, active, rb, len, per_block, vals);
}

// ---------------------------------------------------------------- point access / CSR expansion
__device__ __forceinline__ int64_t value_index(bool per_block, int k, int64_t rb, int64_t nnz_row, int64_t slot, int i,
                                               int j)
{
  // per block: (block_start*k^2) + i*k + j   (femutils/BSRFormat.h:820-829, :160-162)
  // per row:   rb*k^2 + k*slot + i*k*nnz_row + j  (:877-887 with the i-th row offset
  //            i*k*nnz_row; the reference adds k*nnz_row once for every i != 0,
  //            which is only right for k <= 2)
  return per_block ? (rb + slot) * k * k + i * k + j : rb * k * k + (int64_t)i * k * nnz_row + (int64_t)k * slot + j;
}

__global__ void k_bsr_point(int k, bool per_block, const int64_t* __restrict__ rows, const int32_t* __restrict__ cols,
                            double* __restrict__ vals, int32_t row, int32_t col, int op, double v,
                            double* __restrict__ out, int32_t* __restrict__ found)
{
  if (threadIdx.x != 0) return;
  const int32_t br = row / k, bc = col / k;
  const int i = row % k, j = col % k;
  const int64_t rb = rows[br], re = rows[br + 1];
  for (int64_t t = rb; t < re; ++t)
    if (cols[t] == bc) {
      int64_t idx = value_index(per_block, k, rb, re - rb, t - rb, i, j);
      if (op == 1)
        vals[idx] = v;
      else if (op == 2)
        vals[idx] += v;
      *out = vals[idx];
      *found = 1;
      return;
    }
  *found = 0;
}

// One lane per scalar row: row offsets and columns of the scalar expansion.
__global__ void k_expand_rows(int64_t n_brows, int k, const int64_t* __restrict__ rows, int64_t* __restrict__ srows)
{
  int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s > n_brows * k) return;
  if (s == n_brows * k) {
    srows[s] = rows[n_brows] * k * k;
    return;
  }
  int64_t br = s / k;
  int i = (int)(s % k);
  int64_t nnz_row = rows[br + 1] - rows[br];
  srows[s] = rows[br] * k * k + (int64_t)i * k * nnz_row;
}

__global__ void k_expand_cols(int64_t n_brows, int k, bool per_block, const int64_t* __restrict__ rows,
                              const int32_t* __restrict__ cols, const double* __restrict__ vals,
                              int32_t* __restrict__ scols, double* __restrict__ svals)
{
  int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_brows * k) return;
  int64_t br = s / k;
  int i = (int)(s % k);
  int64_t rb = rows[br], nnz_row = rows[br + 1] - rb;
  int64_t out = rb * k * k + (int64_t)i * k * nnz_row;
  for (int64_t t = 0; t < nnz_row; ++t)
    for (int j = 0; j < k; ++j) {
      scols[out + t * k + j] = cols[rb + t] * k + j;
      if (per_block) svals[out + t * k + j] = vals[value_index(true, k, rb, nnz_row, t, i, j)];
    }
}

}  // namespace

bool bsr_point(Bsr& b, int32_t row, int32_t col, int op, double v, double* out)
{
  Ctx& ctx = *b.mesh->ctx;
  const int k = b.nb_dof;
  AFEM_REQUIRE(b.has_sparsity, AFEM_ERR_STATE, "BSR matrix has no sparsity yet");
  AFEM_REQUIRE(row >= 0 && row / k < b.s.n_rows && col >= 0 && col / k < b.s.n_cols, AFEM_ERR_ARG,
               "BSRMatrix: (row,col) out of range");
  DevBuf<double> dv;
  DevBuf<int32_t> df;
  dv.alloc(1);
  df.alloc(1);
  hipLaunchKernelGGL(k_bsr_point, dim3(1), dim3(64), 0, ctx.stream, k, b.order_per_block, b.s.row_ptr.p, b.s.cols.p,
                     b.values.p, row, col, op, v, dv.p, df.p);
  AFEM_LAUNCHED();
  int32_t found = 0;
  double hv = 0.0;
  AFEM_HIP(hipMemcpyAsync(&found, df.p, sizeof(found), hipMemcpyDeviceToHost, ctx.stream));
  AFEM_HIP(hipMemcpyAsync(&hv, dv.p, sizeof(hv), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  if (out) *out = hv;
  return found == 1;
}

void bsr_expand_scalar(Bsr& b, double* vals_out)
{
  Ctx& ctx = *b.mesh->ctx;
  const int k = b.nb_dof;
  const int64_t nbr = b.s.n_rows;
  b.csr_rows.alloc(nbr * k + 1);
  b.csr_cols.alloc(b.s.nnz * k * k);
  hipLaunchKernelGGL(k_expand_rows, dim3((unsigned)((nbr * k + 1 + 255) / 256)), dim3(256), 0, ctx.stream, nbr, k,
                     b.s.row_ptr.p, b.csr_rows.p);
  AFEM_LAUNCHED();
  hipLaunchKernelGGL(k_expand_cols, dim3((unsigned)((nbr * k + 255) / 256)), dim3(256), 0, ctx.stream, nbr, k,
                     b.order_per_block, b.s.row_ptr.p, b.s.cols.p, b.values.p, b.csr_cols.p, vals_out);
  AFEM_LAUNCHED();
}

namespace {
// LDS tile budget per wave (one wave per workgroup): beyond it the global
// accumulation variants run (rows of > ~90 non-zeros, not P1 meshes).
constexpr int64_t kTileLdsMax = 64 * 1024;
// AFEM_ASSEMBLY_WAVES_PER_CU: diagnostic override of the persistent grid size
int occ_override()
{
  static const int v = [] {
    const char* e = variant("AFEM_ASSEMBLY_WAVES_PER_CU");
    return e ? atoi(e) : 0;
  }();
  return v;
}
}  // namespace

// Claim counters of the persistent assembly kernels: one 4-KB slot per
// assembly (up to 4 launches x 8 XCD counters, 128 B apart) from a ring of
// kTicketRing slots zeroed together -- one memset every kTicketRing
// assemblies instead of a fill launch per assembly.  Every launch of an
// assembly is joined to the context stream before the next one starts, so a
// ring reset (stream-ordered) never races a running kernel.
constexpr int64_t kTicketRing = 256, kTicketSlot = 5 * 8 * 16;
unsigned long long* next_tickets(Structure& s, Ctx& ctx)
{
  if (s.tickets.n < kTicketRing * kTicketSlot) {
    s.tickets.alloc(kTicketRing * kTicketSlot);
    s.ticket_gen = 0;
  }
  if (s.ticket_gen % kTicketRing == 0) AFEM_HIP(hipMemsetAsync(s.tickets.p, 0, s.tickets.bytes(), ctx.stream));
  unsigned long long* const t = s.tickets.p + (s.ticket_gen % kTicketRing) * kTicketSlot;
  ++s.ticket_gen;
  return t;
}

// the stencil kernel (every compiled-in signature, stencil_sigs.inc) over s.rec_k
void launch_stencil(const Structure& s, int n_cu, const double* coords, double s_coef, double f_meas, double* vals,
                    double* rhs, int rhs_add, unsigned long long* tk, hipStream_t stream)
{
  static int occ_k = 0;
  static size_t occ_shm = 0;
  static const void* occ_kern = nullptr;
  auto kern = s.canon ? k_assemble_stencil<true, AFEM_STENCIL_PACK> : k_assemble_stencil<false, AFEM_STENCIL_PACK>;
  const size_t shm = (size_t)stencil_tile_bytes(s.k_nodes, stencil_maxw<AFEM_STENCIL_PACK>());
  if (occ_shm != shm || occ_kern != reinterpret_cast<const void*>(kern)) {
    occ_kern = reinterpret_cast<const void*>(kern);
    int q = 0;
    AFEM_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&q, reinterpret_cast<const void*>(kern), 64, shm));
    occ_k = q < 1 ? 1 : q;
    occ_shm = shm;
  }
  const int per_cu = occ_override() > 0 ? occ_override() : occ_k;
  int64_t nblk = (int64_t)n_cu * per_cu;
  if (nblk > s.n_k) nblk = s.n_k < 8 ? 8 : s.n_k;
  hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(64), shm, stream, s.n_k, s.rec_k.p, tk, s.k_nodes, s.perm.p,
                     s.pos_rb.p, s.pos_dl.p, s.strip_u.p, s.snode.p, coords, s_coef, f_meas, vals, rhs, rhs_add, s.cperm.p);
  AFEM_LAUNCHED();
}

int stencil_match(uint64_t pat, int nsteps, int w, const uint8_t* slot32)
{
  static const StencilSig* const table[] = {
#define AFEM_STENCIL_PTR(ID_, SIG_) &SIG_,
    AFEM_STENCIL_SIGS(AFEM_STENCIL_PTR)
#undef AFEM_STENCIL_PTR
  };
  for (int i = 0; i < (int)(sizeof(table) / sizeof(table[0])); ++i) {
    const StencilSig& g = *table[i];
    if (g.pat == pat && g.nsteps == nsteps && g.w == w && memcmp(g.slot, slot32, 32) == 0) return i;
  }
  return -1;
}

void assemble_scalar(Bsr& b, double coef, double f, double* rhs, int rhs_add)
{
  Structure& s = b.s;
  Ctx& ctx = *b.mesh->ctx;
  const int nv = b.mesh->nv;
  AFEM_REQUIRE(b.nb_dof == 1, AFEM_ERR_ARG, "assembleBilinear(P1 Laplacian) needs NB_DOF = 1");
  // generator boxes / slabs: the cell-first cube kernel (cubes.hip)
  if (assemble_cubes(b, coef, f, rhs, rhs_add)) return;
  const int dimc = nv == 4 ? 3 : 2;
  int bucket = -1;
  for (int i = 0; i < 4 && bucket < 0; ++i)
    if (s.max_slice_nodes <= kUcapBuckets[i] && tile_bytes(dimc, 1, kUcapBuckets[i], s.max_slice_w) <= kTileLdsMax)
      bucket = i;
  // K = coef * c0.cb / (6|det|) (tets) or / (2|A2|) (triangles);
  // RHS = f * |K| / nv = f*|det|/24 (tets) or f*|A2|/6 (triangles)
  const double s_coef = (nv == 4) ? coef / 6.0 : coef / 2.0;
  const double f_meas = (nv == 4) ? f / 24.0 : f / 6.0;
  // row strips: the default path (AFEM_ASSEMBLY_STRIPS=0 selects the
  // per-cell incidence kernel, a diagnostic)
  static const bool strips_env = [] {
    const char* e = variant("AFEM_ASSEMBLY_STRIPS");
    return !(e && atoi(e) == 0);
  }();
  if (strips_env && s.strip_ok && s.rec_ok && s.nnz < (int64_t(1) << 32) && s.max_strip_c <= 4 &&
      strip_tile_bytes(dimc, s.max_slice_nodes, s.max_slice_w) <= kTileLdsMax) {
    const size_t shm_g = (size_t)strip_tile_bytes(dimc, s.max_slice_nodes, s.max_slice_w);
    // the uniform tet instance needs neither the column-index table nor the
    // overflow scratch: accumulators + coordinates (<= 13.6 KB: 12 waves per CU)
    const size_t shm_u = (size_t)(8 * 64 * (int64_t)s.max_slice_w + strip_coord_bytes(dimc, s.max_slice_nodes, s.max_slice_w));
    static std::map<std::pair<const void*, size_t>, int> occ_s;
    // AFEM_ASSEMBLY_UNIFORM=0: every slice through the general variant (diagnostic)
    const char* ue = variant("AFEM_ASSEMBLY_UNIFORM");  // read per call: the parity test toggles it
    const int umode = ue ? atoi(ue) : 1;               // 0 off, 1 branches, 2 selects
    const bool uni_env = umode != 0;
    const bool use_uni = uni_env && s.n_uni > 0;
    const int64_t n_mix = use_uni ? s.n_mix : s.n_slices;
    unsigned long long* const tk0 = next_tickets(s, ctx);  // this assembly's claim counters
    auto launch_s = [&](const void* fn, auto kern, int64_t n_list, const SliceRec* list, unsigned long long* tk,
                        size_t shm_s, hipStream_t stream, int ucap = -1, int wcap = -1,
                        const uint8_t* slots = nullptr) {
      if (ucap < 0) ucap = s.max_slice_nodes;
      if (wcap < 0) wcap = s.max_slice_w;
      auto it = occ_s.find({ fn, shm_s });
      if (it == occ_s.end()) {
        int q = 0;
        AFEM_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&q, fn, 64, shm_s));
        it = occ_s.emplace(std::make_pair(fn, shm_s), q < 1 ? 1 : q).first;
      }
      const int per_cu = occ_override() > 0 ? occ_override() : it->second;
      int64_t nblk = (int64_t)ctx.n_cu * per_cu;
      if (nblk > n_list) nblk = n_list < 8 ? 8 : n_list;
      hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(64), shm_s, stream, n_list, list, tk,
                         ucap, wcap, s.perm.p, s.pos_rb.p, s.pos_dl.p, s.strip.p, s.strip_u.p,
                         s.lidx.p, s.snode.p, b.mesh->coords.p, s_coef, f_meas, b.values.p, rhs, rhs_add,
                         reinterpret_cast<const SlotRec*>(slots ? slots : s.uslot.p), s.cperm.p);
    };
    // canonical structures (compact strips, <= 16 slots: sparsity.hip) run the
    // PERM instances; no other instance knows the slot map
    // (the uniform slices through the select instance, UMODE 2, same bits: the
    // 3-waves-per-SIMD branch instance has no registers for the map)
#define AFEM_SK(NV_, C_, W_, U_) \
  (s.canon ? k_assemble_strip<NV_, C_, W_, (U_ == 1 ? 2 : U_), true> : k_assemble_strip<NV_, C_, W_, U_, false>)
#define AFEM_SKF(NV_, C_, W_, U_) reinterpret_cast<const void*>(AFEM_SK(NV_, C_, W_, U_))
    AFEM_REQUIRE(!s.canon || (nv == 4 && s.max_strip_c <= 2 && s.max_slice_w <= 16 && s.n_mb == 0), AFEM_ERR_STATE,
                 "canonical structure beyond the compact strip instances");
    const SliceRec* list_m = use_uni ? s.rec_m.p : s.rec_all.p;
#define AFEM_STRIP_K(NV_, C_, W_, U_, N_, L_, T_, SHM_, ST_) \
  launch_s(AFEM_SKF(NV_, C_, W_, U_), AFEM_SK(NV_, C_, W_, U_), N_, L_, T_, SHM_, ST_)
    const bool small = s.max_strip_c <= 2 && s.max_slice_w <= 16;
    if (nv == 4 && uni_env) {
      // uniform slices on the context stream; the general-instance slices in
      // two lists (compact / big: sparsity.hip) with their own LDS tiles.  With
      // uniform slices the general lists run on the side stream beside the
      // uniform instance (fork / join through events): their launch and tail
      // hide under the large kernel; without (unstructured meshes) the
      // compact list runs on the context stream and the big one beside it.
      const bool has_u = s.n_uni > 0;
      // stencil split (AFEM_ASSEMBLY_STENCIL=0: the whole uniform list through the
      // uniform instance, diagnostic): the signature's slices on the context
      // stream, the other uniform slices through the uniform instance beside them
      const char* ke = variant("AFEM_ASSEMBLY_STENCIL");  // read per call: the parity test toggles it
      const bool use_k = has_u && umode == 1 && s.n_k > 0 && !(ke && atoi(ke) == 0);
      // with the stencil split every list runs on the context stream, the small
      // ones first: beside the stencil kernel's persistent grid a side-stream
      // launch only gets CUs as its waves retire (its kernel time stretches to
      // the whole assembly), one after the other the kernel times add up to the
      // assembly time (AFEM_ASSEMBLY_SIDE=1: side stream, diagnostic)
      const char* se = variant("AFEM_ASSEMBLY_SIDE");
      const int side_mode = se ? atoi(se) : 0;
      const bool serial_k = use_k && side_mode != 1;
      // AFEM_ASSEMBLY_SIDE=2: the small lists first on the context stream, the
      // stencil kernel on the side stream right after (forked before them), so
      // the small lists' waves are dispatched first and the stencil grid fills
      // the rest of the chip beside them
      const bool k_side = use_k && side_mode == 2 && (s.n_ms > 0 || s.n_mb > 0);
      // without uniform slices: the compact list, then the big one, on the context
      // stream (AFEM_ASSEMBLY_BIG=2, the default); =1 the big list first; =0 the big
      // list beside the compact one on the side stream.  Refined L-shape-3D (r05au,
      // one process): 1.289 / 1.289 / 1.310 ms -- side by side, the two persistent
      // grids share the chip and the big one's tail sets the end
      const char* bge = variant("AFEM_ASSEMBLY_BIG");
      const int big_mode = has_u ? 0 : (bge ? atoi(bge) : 2);
      const bool fork = k_side || (!serial_k && ((has_u && (s.n_ms > 0 || s.n_mb > 0 || (use_k && s.n_ur > 0))) ||
                                                 (!has_u && big_mode == 0 && s.n_ms > 0 && s.n_mb > 0)));
      hipStream_t side = ctx.stream;
      if (fork) {
        side = ctx.side();
        AFEM_HIP(hipEventRecord(ctx.ev_fork, ctx.stream));
        AFEM_HIP(hipStreamWaitEvent(side, ctx.ev_fork, 0));
      }
      const int ms_w = 16;
      const size_t shm_ms = (size_t)strip_tile_bytes(dimc, s.ms_nodes, ms_w);
      const size_t shm_mb = (size_t)strip_tile_bytes(dimc, s.mb_nodes, s.mb_w);
      const bool mb_ok = s.mb_w <= 32 && s.n_mb >= 0 && shm_mb <= kTileLdsMax;
      AFEM_REQUIRE(s.n_mb == 0 || (mb_ok && s.max_strip_c <= 4), AFEM_ERR_STATE, "strip lists exceed the kernels");
      hipStream_t s_ms = has_u && !serial_k ? side : ctx.stream;
      hipStream_t s_mb = has_u && !serial_k ? side : (s.n_ms > 0 && !serial_k && big_mode == 0 ? side : ctx.stream);
      auto launch_mb = [&]() {
        if (s.n_mb > 0)
          launch_s(reinterpret_cast<const void*>(&k_assemble_strip<4, 4, 32, 0>), k_assemble_strip<4, 4, 32, 0>, s.n_mb,
                   s.rec_mb.p, tk0 + 256, shm_mb, s_mb, s.mb_nodes, s.mb_w);
      };
      if (big_mode == 1) launch_mb();
      // AFEM_ASSEMBLY_LOCAL=1: the compact list's slices of <= 256 nodes through the
      // local-index-stream instance (UMODE 3: no column-index table, no dependent
      // LDS read per step), the rest through UMODE 0.  Measured on the refined
      // L-shape (r04h): 1.458 vs 1.413 ms -- 43 % of its compact slices have more
      // than 256 nodes, the two launches run one after the other, and the bank
      // conflicts stay (4.0e7 + 6.0e7 cycles: not the column-index reads)
      const char* le = variant("AFEM_ASSEMBLY_LOCAL");
      const int64_t n_loc = (le && atoi(le) == 1 && !s.canon) ? s.n_msl : 0;
      if (n_loc > 0) {
        const size_t shm_l = (size_t)strip_tile_bytes(dimc, s.msl_nodes, ms_w);
        launch_s(reinterpret_cast<const void*>(&k_assemble_strip<4, 2, 16, 3>), k_assemble_strip<4, 2, 16, 3>, n_loc,
                 s.rec_ms.p, tk0 + 512, shm_l, s_ms, s.msl_nodes, ms_w);
      }
      if (s.n_ms > n_loc)
        launch_s(AFEM_SKF(4, 2, 16, 0), AFEM_SK(4, 2, 16, 0), s.n_ms - n_loc,
                 s.rec_ms.p + n_loc, tk0 + 128, shm_ms, s_ms, s.ms_nodes, ms_w);
      if (big_mode != 1) launch_mb();
      if (use_k) {
        if (s.n_ur > 0) {
          const size_t shm_ur = (size_t)(8 * 64 * (int64_t)s.ur_w + strip_coord_bytes(dimc, s.ur_nodes, s.ur_w));
          launch_s(AFEM_SKF(4, 2, 16, 1), AFEM_SK(4, 2, 16, 1),
                   s.n_ur, s.rec_ur.p, tk0, shm_ur, side, s.ur_nodes, s.ur_w, s.urslot.p);
        }
        launch_stencil(s, ctx.n_cu, b.mesh->coords.p, s_coef, f_meas, b.values.p, rhs, rhs_add,
                       tk0 + 384, k_side ? side : ctx.stream);
      }
      else if (has_u) {
        const size_t shm_uu = (size_t)(8 * 64 * (int64_t)s.u_w + strip_coord_bytes(dimc, s.u_nodes, s.u_w));
        if (umode == 2)
          launch_s(AFEM_SKF(4, 2, 16, 2), AFEM_SK(4, 2, 16, 2),
                   s.n_uni, s.rec_u.p, tk0, shm_uu, ctx.stream, s.u_nodes, s.u_w);
        else
          launch_s(AFEM_SKF(4, 2, 16, 1), AFEM_SK(4, 2, 16, 1),
                   s.n_uni, s.rec_u.p, tk0, shm_uu, ctx.stream, s.u_nodes, s.u_w);
      }
      AFEM_LAUNCHED();
      if (fork) {
        AFEM_HIP(hipEventRecord(ctx.ev_join, side));
        AFEM_HIP(hipStreamWaitEvent(ctx.stream, ctx.ev_join, 0));
      }
    }
    else if (nv == 4) {
      // every slice through the general instance (AFEM_ASSEMBLY_UNIFORM=0, diagnostic)
      const bool fork = use_uni && n_mix > 0;
      hipStream_t ms = ctx.stream;
      if (fork) {
        ms = ctx.side();
        AFEM_HIP(hipEventRecord(ctx.ev_fork, ctx.stream));
        AFEM_HIP(hipStreamWaitEvent(ms, ctx.ev_fork, 0));
      }
      if (small) {
        if (n_mix > 0) AFEM_STRIP_K(4, 2, 16, 0, n_mix, list_m, tk0 + 128, shm_g, ms);
        if (use_uni && umode == 2) AFEM_STRIP_K(4, 2, 16, 2, s.n_uni, s.rec_u.p, tk0, shm_u, ctx.stream);
        else if (use_uni) AFEM_STRIP_K(4, 2, 16, 1, s.n_uni, s.rec_u.p, tk0, shm_u, ctx.stream);
      }
      else {
        if (n_mix > 0) AFEM_STRIP_K(4, 4, 32, 0, n_mix, list_m, tk0 + 128, shm_g, ms);
        if (use_uni) AFEM_STRIP_K(4, 4, 32, 1, s.n_uni, s.rec_u.p, tk0, shm_u, ctx.stream);
      }
      AFEM_LAUNCHED();
      if (fork) {
        AFEM_HIP(hipEventRecord(ctx.ev_join, ms));
        AFEM_HIP(hipStreamWaitEvent(ctx.stream, ctx.ev_join, 0));
      }
    }
    else {
      if (small) AFEM_STRIP_K(3, 2, 16, 0, s.n_slices, s.rec_all.p, tk0 + 128, shm_g, ctx.stream);
      else AFEM_STRIP_K(3, 4, 32, 0, s.n_slices, s.rec_all.p, tk0 + 128, shm_g, ctx.stream);
    }
#undef AFEM_STRIP_K
#undef AFEM_SK
#undef AFEM_SKF
    AFEM_LAUNCHED();
    b.last_kernel = AFEM_KERNEL_STRIP;
    return;
  }
  AFEM_REQUIRE(!s.canon, AFEM_ERR_STATE, "a canonical structure needs the strip kernels");
  // register-resident incidence groups per lane / fixed write-back width
  const int max_groups = s.max_slice_k >> 2;
  const int prof = (max_groups <= 6 && s.max_slice_w <= 16) ? 0 : (max_groups <= 16 ? 1 : -1);
  const dim3 grid((unsigned)s.n_slices), blk(64);
  if (bucket < 0 || prof < 0) {
    if (nv == 4)
      hipLaunchKernelGGL(k_assemble_p1_global<4>, grid, blk, 0, ctx.stream, s.perm.p, s.row_ptr.p, s.cols.p, s.inc.p,
                         s.inc_slice_ptr.p, s.inc_slice_k.p, b.mesh->coords.p, s_coef, f_meas, b.values.p, rhs, rhs_add);
    else
      hipLaunchKernelGGL(k_assemble_p1_global<3>, grid, blk, 0, ctx.stream, s.perm.p, s.row_ptr.p, s.cols.p, s.inc.p,
                         s.inc_slice_ptr.p, s.inc_slice_k.p, b.mesh->coords.p, s_coef, f_meas, b.values.p, rhs, rhs_add);
    AFEM_LAUNCHED();
    b.last_kernel = AFEM_KERNEL_GLOBAL;
    return;
  }
  const size_t shm = (size_t)tile_bytes(dimc, 1, kUcapBuckets[bucket], s.max_slice_w);
  // persistent grid: as many single-wave workgroups as the LDS tile and the
  // registers let reside at once, each walking a contiguous chunk of slices
  // (occupancy queried once per (kernel, LDS size); kept off the launch path)
  static std::map<std::pair<const void*, size_t>, int> occ;
  auto launch = [&](const void* fn, auto kern) {
    auto it = occ.find({ fn, shm });
    if (it == occ.end()) {
      int q = 0;
      AFEM_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&q, fn, 64, shm));
      it = occ.emplace(std::make_pair(fn, shm), q < 1 ? 1 : q).first;
    }
    const int per_cu = occ_override() > 0 ? occ_override() : it->second;
    const int64_t waves = (int64_t)ctx.n_cu * per_cu;
    const int64_t chunk = (s.n_slices + waves - 1) / waves;
    const int64_t nblk = (s.n_slices + chunk - 1) / chunk;
    hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(64), shm, ctx.stream, s.n_slices, chunk,
                       s.max_slice_nodes, s.max_slice_w, s.inc_pad_off, s.perm.p, s.row_ptr.p, s.inc.p,
                       s.inc_slice_ptr.p, s.inc_slice_k.p, s.slice_w.p, s.lidx_ptr.p, s.lidx.p, s.snode_ptr.p,
                       s.snode.p, b.mesh->coords.p, s_coef, f_meas, b.values.p, rhs, rhs_add);
  };
#define AFEM_ASM_K(NV_, U_, G_, W_) launch(reinterpret_cast<const void*>(&k_assemble_p1<NV_, U_, G_, W_>), k_assemble_p1<NV_, U_, G_, W_>)
#define AFEM_ASM_LAUNCH(NV_, U_)                \
  do {                                          \
    if (prof == 0) AFEM_ASM_K(NV_, U_, 6, 16);  \
    else AFEM_ASM_K(NV_, U_, 16, 32);           \
  } while (0)
  if (nv == 4) {
    switch (bucket) {
      case 0: AFEM_ASM_LAUNCH(4, 257); break;
      case 1: AFEM_ASM_LAUNCH(4, 513); break;
      case 2: AFEM_ASM_LAUNCH(4, 1025); break;
      default: AFEM_ASM_LAUNCH(4, 2049);
    }
  }
  else {
    switch (bucket) {
      case 0: AFEM_ASM_LAUNCH(3, 257); break;
      case 1: AFEM_ASM_LAUNCH(3, 513); break;
      case 2: AFEM_ASM_LAUNCH(3, 1025); break;
      default: AFEM_ASM_LAUNCH(3, 2049);
    }
  }
#undef AFEM_ASM_K
#undef AFEM_ASM_LAUNCH
  AFEM_LAUNCHED();
  b.last_kernel = AFEM_KERNEL_SLICE_TILE;
}

bool assembly_uses_lds(const Bsr& b)
{
  const int nacc = b.nb_dof * b.nb_dof;
  const int dimc = b.mesh->nv == 4 ? 3 : 2;
  if (nacc == 1) {
    for (int u : kUcapBuckets)
      if (b.s.max_slice_nodes <= u && tile_bytes(dimc, 1, u, b.s.max_slice_w) <= kTileLdsMax) return true;
    return false;
  }
  return tile_bytes(dimc, nacc, b.s.max_slice_nodes, b.s.max_slice_w) <= kTileLdsMax;
}

void assemble_elasticity_tet(Bsr& b, double lambda, double mu2, double c0, const double* f, double* rhs, int rhs_add)
{
  Structure& s = b.s;
  Ctx& ctx = *b.mesh->ctx;
  AFEM_REQUIRE(b.nb_dof == 3 && b.mesh->nv == 4, AFEM_ERR_NOT_IMPL,
               "block-3 P1 elasticity assembly needs NB_DOF = 3 on tetrahedra");
  const double fx = f ? f[0] : 0.0, fy = f ? f[1] : 0.0, fz = f ? f[2] : 0.0;
  const int64_t shm_old = 3 * 8 * 64 * (int64_t)s.max_slice_w + ((24 * (int64_t)s.max_slice_nodes + 15) & ~int64_t(15)) +
                          2 * 64 * (int64_t)s.max_slice_w;
  // unstructured meshes: rows up to 32 slots, slices beyond 256 nodes, strips up to 64 steps
  const size_t shm_big = (size_t)elast_tile_bytes(s.max_slice_nodes, s.max_slice_w);
  const bool big_ok = s.strip_ok && s.rec_ok && s.max_strip_c <= 4 && s.max_slice_w <= 32 &&
                      shm_big <= 160 * 1024 && s.nnz * 9 < (int64_t(1) << 40);
  const bool fits_small = s.strip_ok && s.max_slice_w <= 16 && shm_old <= 160 * 1024;
  const char* be = variant("AFEM_ELAST_BIG");  // 0: the global kernel instead (diagnostic)
  if (!fits_small && big_ok && !(be && atoi(be) == 0)) {
    // three lists (sparsity.hip): uniform and compact slices (<= 16 slots, <= 32
    // steps, <= 352 nodes) through the <2, 16> instance with a tile sized by
    // their own maxima, the big ones through <4, 32> beside them on the side
    // stream: the few large slices no longer set the LDS tile (and the
    // occupancy) of all
    static std::map<std::pair<const void*, size_t>, int> occ_big;
    unsigned long long* const tk0 = next_tickets(s, ctx);  // this assembly's claim counters
    auto launch = [&](const void* fn, auto kern, int64_t n_list, const SliceRec* list, unsigned long long* tk,
                      int ucap, int wcap, hipStream_t st) {
      const size_t shm = (size_t)elast_tile_bytes(ucap, wcap);
      auto it = occ_big.find({ fn, shm });
      if (it == occ_big.end()) {
        int q = 0;
        AFEM_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&q, fn, 64, shm));
        it = occ_big.emplace(std::make_pair(fn, shm), q < 1 ? 1 : q).first;
      }
      const int64_t n_items = 3 * n_list;
      int64_t nblk = (int64_t)ctx.n_cu * it->second;
      if (nblk > n_items) nblk = n_items < 8 ? 8 : n_items;
      hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(64), shm, st, n_items, list, tk, ucap, wcap,
                         b.order_per_block, s.perm.p, s.pos_rb.p, s.pos_dl.p, s.strip.p, s.lidx.p, s.snode.p,
                         b.mesh->coords.p, lambda, 0.5 * mu2, c0, fx, fy, fz, b.values.p, f ? rhs : nullptr, rhs_add);
      AFEM_LAUNCHED();
    };
    const int c_nodes = std::max(s.u_nodes, s.ms_nodes);
    const bool split = s.n_mb < s.n_slices && elast_tile_bytes(c_nodes, 16) <= 160 * 1024 &&
                       elast_tile_bytes(s.mb_nodes, s.mb_w) <= 160 * 1024;
    if (!split) {
      launch(reinterpret_cast<const void*>(&k_assemble_elast_strip<4, 32, 0, true>), k_assemble_elast_strip<4, 32, 0, true>,
             s.n_slices, s.rec_all.p, tk0, s.max_slice_nodes, s.max_slice_w, ctx.stream);
    }
    else {
      const bool fork = s.n_mb > 0;
      hipStream_t side = ctx.stream;
      if (fork) {
        side = ctx.side();
        AFEM_HIP(hipEventRecord(ctx.ev_fork, ctx.stream));
        AFEM_HIP(hipStreamWaitEvent(side, ctx.ev_fork, 0));
      }
      if (s.n_mb > 0)
        launch(reinterpret_cast<const void*>(&k_assemble_elast_strip<4, 32, 0, true>),
               k_assemble_elast_strip<4, 32, 0, true>, s.n_mb, s.rec_mb.p, tk0 + 256, s.mb_nodes, s.mb_w, side);
      if (s.n_ms > 0)
        launch(reinterpret_cast<const void*>(&k_assemble_elast_strip<2, 16, 0, true>),
               k_assemble_elast_strip<2, 16, 0, true>, s.n_ms, s.rec_ms.p, tk0 + 128, c_nodes, 16, ctx.stream);
      if (s.n_uni > 0)
        launch(reinterpret_cast<const void*>(&k_assemble_elast_strip<2, 16, 0, true>),
               k_assemble_elast_strip<2, 16, 0, true>, s.n_uni, s.rec_u.p, tk0, c_nodes, 16, ctx.stream);
      if (fork) {
        AFEM_HIP(hipEventRecord(ctx.ev_join, side));
        AFEM_HIP(hipStreamWaitEvent(ctx.stream, ctx.ev_join, 0));
      }
    }
    b.last_kernel = AFEM_KERNEL_ELAST3_BIG;
    return;
  }
  if (!fits_small) {
    // no row strips (high-valence nodes) or rows / slices too large for any LDS tile
    hipLaunchKernelGGL(k_assemble_elast_tet_global, dim3((unsigned)(3 * s.n_slices)), dim3(64), 0, ctx.stream,
                       b.order_per_block, s.perm.p, s.row_ptr.p, s.cols.p, s.inc.p, s.inc_slice_ptr.p, s.inc_slice_k.p,
                       b.mesh->coords.p, lambda, 0.5 * mu2, c0, fx, fy, fz, b.values.p, f ? rhs : nullptr, rhs_add);
    AFEM_LAUNCHED();
    b.last_kernel = AFEM_KERNEL_ELAST3_GLOBAL;
    return;
  }
  // one workgroup (three waves) per slice (AFEM_ELAST_WG=0: one wave per (slice, component), diagnostic)
  const char* we = variant("AFEM_ELAST_WG");
  const bool use_wg = !(we && atoi(we) == 0);
  const int64_t ucap2 = (s.max_slice_nodes + 1) & ~int64_t(1);  // 16-B aligned column-index table
  if (use_wg && s.rec_ok && s.max_strip_c <= 2 && s.max_slice_w <= 16 && s.max_slice_nodes <= 256 &&
      s.nnz * 9 < (int64_t(1) << 40) && elast_wg_bytes(ucap2, s.max_slice_w) <= 160 * 1024) {
    const size_t shm = (size_t)elast_wg_bytes(ucap2, s.max_slice_w);
    static std::map<std::pair<const void*, size_t>, int> occ_wg;
    const char* ue = variant("AFEM_ASSEMBLY_UNIFORM");
    const bool use_uni = !(ue && atoi(ue) == 0) && s.n_uni > 0;
    // stencil split (AFEM_ASSEMBLY_STENCIL=0: the whole uniform list through the uniform instance)
    const char* ke = variant("AFEM_ASSEMBLY_STENCIL");
    const bool use_k = use_uni && s.n_k0 > 0 && !(ke && atoi(ke) == 0);
    unsigned long long* const tk0 = next_tickets(s, ctx);  // this assembly's claim counters
    auto launch = [&](const void* fn, auto kern, int64_t n_items, const SliceRec* list, unsigned long long* tk,
                      const uint8_t* slots = nullptr) {
      auto it = occ_wg.find({ fn, shm });
      if (it == occ_wg.end()) {
        int q = 0;
        AFEM_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&q, fn, 192, shm));
        it = occ_wg.emplace(std::make_pair(fn, shm), q < 1 ? 1 : q).first;
      }
      // AFEM_ELAST_WG_OCC: workgroups per CU of the persistent grid (diagnostic; default the occupancy)
      const char* oe = variant("AFEM_ELAST_WG_OCC");
      const int occ_wg_cu = oe && atoi(oe) > 0 ? std::min(atoi(oe), it->second) : it->second;
      int64_t nblk = (int64_t)ctx.n_cu * occ_wg_cu;
      if (nblk > n_items) nblk = n_items < 8 ? 8 : n_items;
      hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(192), shm, ctx.stream, n_items, list, tk, (int)ucap2,
                         s.max_slice_w, b.order_per_block, s.perm.p, s.pos_rb.p, s.pos_dl.p, s.strip.p, s.lidx.p,
                         s.snode.p, b.mesh->coords.p, lambda, 0.5 * mu2, c0, fx, fy, fz, b.values.p, f ? rhs : nullptr,
                         rhs_add, s.strip_u.p, reinterpret_cast<const SlotRec*>(slots ? slots : s.uslot.p));
      AFEM_LAUNCHED();
    };
    if (use_k) {
      launch(reinterpret_cast<const void*>(&k_assemble_elast_wg<2, 16, 3>), k_assemble_elast_wg<2, 16, 3>, s.n_k0,
             s.rec_k0.p, tk0 + 384);
      if (s.n_u1 > 0)
        launch(reinterpret_cast<const void*>(&k_assemble_elast_wg<2, 16, 1>), k_assemble_elast_wg<2, 16, 1>, s.n_u1,
               s.rec_u1.p, tk0, s.u1slot.p);
    }
    else if (use_uni)
      launch(reinterpret_cast<const void*>(&k_assemble_elast_wg<2, 16, 1>), k_assemble_elast_wg<2, 16, 1>, s.n_uni,
             s.rec_u.p, tk0);
    const int64_t n_mix = use_uni ? s.n_mix : s.n_slices;
    if (n_mix > 0)
      launch(reinterpret_cast<const void*>(&k_assemble_elast_wg<2, 16, 0>), k_assemble_elast_wg<2, 16, 0>, n_mix,
             use_uni ? s.rec_m.p : s.rec_all.p, tk0 + 128);
    b.last_kernel = AFEM_KERNEL_ELAST3_WG;
    return;
  }
  // persistent pipelined kernel, one wave per (slice, component) (AFEM_ELAST_STRIP=0: the
  // one-wave-per-item kernel, diagnostic)
  const char* ee = variant("AFEM_ELAST_STRIP");
  const bool use_new = !(ee && atoi(ee) == 0);
  if (use_new && s.rec_ok && s.max_strip_c <= 2 && s.max_slice_w <= 16 && s.max_slice_nodes <= 256 &&
      s.nnz * 9 < (int64_t(1) << 40)) {
    const size_t shm2 = (size_t)elast_tile_bytes(s.max_slice_nodes, s.max_slice_w);
    static std::map<std::pair<const void*, size_t>, int> occ;
    // AFEM_ASSEMBLY_UNIFORM=0: every slice through the general instance (diagnostic)
    const char* ue = variant("AFEM_ASSEMBLY_UNIFORM");
    const bool use_uni = !(ue && atoi(ue) == 0) && s.n_uni > 0;
    unsigned long long* const tk0 = next_tickets(s, ctx);  // this assembly's claim counters
    auto launch = [&](const void* fn, auto kern, int64_t n_items, const SliceRec* list, unsigned long long* tk) {
      auto it = occ.find({ fn, shm2 });
      if (it == occ.end()) {
        int q = 0;
        AFEM_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&q, fn, 64, shm2));
        it = occ.emplace(std::make_pair(fn, shm2), q < 1 ? 1 : q).first;
      }
      int64_t nblk = (int64_t)ctx.n_cu * it->second;
      if (nblk > n_items) nblk = n_items < 8 ? 8 : n_items;
      hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(64), shm2, ctx.stream, n_items, list, tk, s.max_slice_nodes,
                         s.max_slice_w, b.order_per_block, s.perm.p, s.pos_rb.p, s.pos_dl.p, s.strip.p, s.lidx.p,
                         s.snode.p, b.mesh->coords.p, lambda, 0.5 * mu2, c0, fx, fy, fz, b.values.p, f ? rhs : nullptr, rhs_add);
      AFEM_LAUNCHED();
    };
    if (use_uni)
      launch(reinterpret_cast<const void*>(&k_assemble_elast_strip<2, 16, 1>), k_assemble_elast_strip<2, 16, 1>,
             3 * s.n_uni, s.rec_u.p, tk0);
    const int64_t n_mix = use_uni ? s.n_mix : s.n_slices;
    if (n_mix > 0)
      launch(reinterpret_cast<const void*>(&k_assemble_elast_strip<2, 16, 0>), k_assemble_elast_strip<2, 16, 0>,
             3 * n_mix, use_uni ? s.rec_m.p : s.rec_all.p, tk0 + 128);
    b.last_kernel = AFEM_KERNEL_ELAST3_STRIP;
    return;
  }
  hipLaunchKernelGGL(k_assemble_elast_tet<16>, dim3((unsigned)(3 * s.n_slices)), dim3(64), (size_t)shm_old, ctx.stream,
                     s.max_slice_nodes, s.max_slice_w, b.order_per_block, s.perm.p, s.row_ptr.p, s.strip.p,
                     s.strip_ptr.p, s.strip_n.p, s.dslot.p, s.slice_w.p, s.lidx_ptr.p, s.lidx.p, s.snode_ptr.p,
                     s.snode.p, b.mesh->coords.p, lambda, 0.5 * mu2, c0, fx, fy, fz, b.values.p, f ? rhs : nullptr, rhs_add);
  AFEM_LAUNCHED();
  b.last_kernel = AFEM_KERNEL_ELAST3_ITEM;
}

void assemble_elasticity_tri(Bsr& b, double lambda, double mu2)
{
  Structure& s = b.s;
  Ctx& ctx = *b.mesh->ctx;
  AFEM_REQUIRE(b.nb_dof == 2 && b.mesh->nv == 3, AFEM_ERR_NOT_IMPL,
               "P1 elasticity assembly is implemented for NB_DOF = 2 on triangles (the reference's elasticity module)");
  const int64_t shm = tile_bytes(2, 4, s.max_slice_nodes, s.max_slice_w);
  const bool lds = shm <= kTileLdsMax;
  const dim3 grid((unsigned)s.n_slices), blk(64);
#define AFEM_EL_ARGS s.max_slice_nodes, s.max_slice_w, s.run, b.order_per_block, s.perm.p, s.row_ptr.p, s.cols.p, s.inc.p, \
                     s.inc_slice_ptr.p, s.inc_slice_k.p, s.slice_w.p, s.lidx_ptr.p, s.lidx.p, s.snode_ptr.p,         \
                     s.snode.p, b.mesh->coords.p, lambda, mu2, b.values.p
  if (lds)
    hipLaunchKernelGGL(k_assemble_elast_tri<true>, grid, blk, (size_t)shm, ctx.stream, AFEM_EL_ARGS);
  else
    hipLaunchKernelGGL(k_assemble_elast_tri<false>, grid, blk, 0, ctx.stream, AFEM_EL_ARGS);
#undef AFEM_EL_ARGS
  AFEM_LAUNCHED();
  b.last_kernel = AFEM_KERNEL_ELAST2;
}

}  // namespace afem
