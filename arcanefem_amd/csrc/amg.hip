// Algebraic multigrid preconditioner for the PCG (afem_solver_opts.amg) on
// systems that are NOT a structured Kuhn box -- Gmsh meshes, caller arrays,
// anything the geometric hierarchy of multigrid.hip does not cover.  The
// reference's GPU solve is Hypre PCG + BoomerAMG on any mesh
// (femutils/HypreDoFLinearSystem.cc:686-742); this is an aggregation AMG built
// from the assembled CSR alone, on the device, deterministic bit for bit:
//  * strength: a_ij is strong when |a_ij| >= theta sqrt(|a_ii a_jj|)
//    (AFEM_AMG_THETA, default 0.05); constraint rows (the PCG's `cons` flags:
//    penalty / eliminated rows) and rows without a positive diagonal are
//    outside the graph;
//  * aggregation: a maximal independent set of the strength graph at distance
//    2 (AFEM_AMG_HOPS0 / AFEM_AMG_HOPS: the fine / coarse levels) by hashed
//    priorities (Luby-style rounds of
//    max propagation over (state, hash(i), i) tuples: no atomics, the same set
//    on every run); every root starts an aggregate, every other node joins the
//    neighbouring root with the largest tuple (distance 2: the aggregate of
//    its largest joined neighbour);
//  * prolongation: piecewise constant on the aggregates (unsmoothed), R = P^T,
//    coarse operator A_c = P^T A P: every strong-graph non-zero (i, j) keyed
//    by (agg i, agg j), radix-sorted (stable), each key run summed by one
//    thread in the CSR order -- fixed summation order;
//  * cycle: V(nu, nu) with damped Jacobi, omega = 4 / (3 lambda_max(D^-1 A))
//    per level (8 power iterations from a signed hashed vector, +10 %: 20 cost
//    10 ms more setup and 70 instead of 64 PCG iterations, r06bm), the
//    coarse correction scaled by AFEM_AMG_SCALE (default 1.7: unsmoothed
//    aggregation under-corrects; 142 -> 92 iterations at 1.7, r05y); the
//    cycle's products on fp32 copies of the values (AFEM_AMG_F32: 2 every level,
//    the default; 1 the fine level, whose product has the residual / Jacobi
//    epilogue fused, k_amg_f32; 0 fp64 -- the fine level then through the PCG's
//    own SpMV plan); the PCG's own product is always fp64; coarsest level (<= 1024 rows,
//    AFEM_AMG_DENSE) inverted densely (host Cholesky at setup), else 24
//    Jacobi sweeps;
//  * K-cycle (AFEM_AMG_KCYCLE, default 2): levels 1..k solve their coarse
//    problem by two flexible-CG steps preconditioned by the cycle below
//    (Notay & Vassilevski), the step weights computed on the device -- the
//    Krylov weights replace the 1.7 overcorrection there;
//  * constraint rows are taken out of the cycle as in multigrid.hip:
//    z = F V(F r) + C D^-1 r (one rank: the mask fused with the first sweep and
//    the fix with the last, AFEM_AMG_FUSE).
// Several ranks (a halo attached): the levels stay distributed -- each rank
// aggregates its own rows, the coarse ghost columns and halo follow from the
// fine halo (build_dist_coarse) -- until the global coarse size is below
// AFEM_AMG_GATHER rows, then one level is gathered on every rank (all-reduce of
// its COO) and the hierarchy below it is the one-rank one, built identically
// everywhere; the Hypre BoomerAMG role on the Arcane communicator
// (femutils/HypreDoFLinearSystem.cc:399-404, 686-742).  The V-cycle is symmetric (an SPD
// preconditioner); the K-cycle is a nonlinear one: the PCG then takes the
// flexible (Polak-Ribiere) beta, -(z.q)/(p.q) (linear_system.hip k_cg_dir_flex;
// tested against the Jacobi-PCG and the plain V-cycle, test_amg_kcycle).
#include "afem_internal.hpp"

#include <hipcub/hipcub.hpp>

#include "kcycle.hpp"

#include <algorithm>
#include <cmath>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

namespace afem {

namespace {

inline unsigned grid_for(int64_t n, int threads) { return (unsigned)((n + threads - 1) / threads); }
constexpr int kDense = 1024;     // rows of a coarsest level inverted densely (AFEM_AMG_DENSE)
constexpr int kMaxLevels = 16;
constexpr int kCoarseSweeps = 24;
constexpr int kPowerIts = 8;    // per level (AFEM_AMG_POWER_ITS)
constexpr int kVec = 1024;       // grid of the vector kernels

// ------------------------------------------------------------------ kernels

__global__ void k_amg_diag(int64_t n, const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
                           const double* __restrict__ v, const uint8_t* __restrict__ cons, double* __restrict__ diag,
                           uint8_t* __restrict__ in)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double d = 0.0;
  for (int64_t k = rp[i]; k < rp[i + 1]; ++k)
    if (ci[k] == i) d += v[k];
  diag[i] = d;
  in[i] = (d > 0.0 && !(cons && cons[i])) ? 1 : 0;
}

__device__ __forceinline__ uint32_t amg_hash(uint32_t x)
{
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// tuple (state, hash, index): state 2 root, 1 undecided, 0 out / outside the graph
__global__ void k_amg_tuple_init(int64_t n, const uint8_t* __restrict__ in, uint64_t* __restrict__ t)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  t[i] = in[i] ? (1ull << 62) | (uint64_t)(amg_hash((uint32_t)i) >> 2) << 32 | (uint64_t)(uint32_t)i : 0ull;
}

__device__ __forceinline__ bool amg_strong(double aij, double di, double dj, double theta)
{
  return fabs(aij) >= theta * sqrt(di * dj);
}

// strong[k] = 1 when non-zero k = (i, j) is an edge of the strength graph
// (8 lanes per row: the row's columns and values read coalesced)
__global__ __launch_bounds__(256) void k_amg_strength(int64_t n, const int64_t* __restrict__ rp,
                                                      const int32_t* __restrict__ ci, const double* __restrict__ v,
                                                      const double* __restrict__ diag,
                                                      const uint8_t* __restrict__ in, double theta,
                                                      uint8_t* __restrict__ strong)
{
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3;
  const int l = threadIdx.x & 7;
  if (i >= n) return;
  const bool ii = in[i];
  const double di = diag[i];
  for (int64_t k = rp[i] + l; k < rp[i + 1]; k += 8) {
    const int32_t j = ci[k];
    strong[k] = (ii && j != i && j >= 0 && j < n && in[j] && amg_strong(v[k], di, diag[j], theta)) ? 1 : 0;
  }
}

// m[i] = max(t[i], t[j] for strong neighbours j); 8 lanes per row.  gate (the
// round's last hop): only the undecided rows' maxima are read (k_amg_mis_update),
// the others are skipped; those rows mark (mark[i] = mark[j] = markv) the rows
// whose first-hop maxima they read, and the next round's first hop computes only
// the rows marked for it (relg[i] == relv: the undecided set only shrinks, so
// they are all the next round reads)
__global__ __launch_bounds__(256) void k_amg_maxprop(int64_t n, const int64_t* __restrict__ rp,
                                                     const int32_t* __restrict__ ci,
                                                     const uint8_t* __restrict__ strong,
                                                     const uint64_t* __restrict__ t, uint64_t* __restrict__ m,
                                                     const uint64_t* __restrict__ gate, const uint8_t* __restrict__ relg,
                                                     int relv, uint8_t* __restrict__ mark, int markv)
{
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3;
  const int l = threadIdx.x & 7;
  if (gate && i < n && (gate[i] >> 62) != 1) return;
  if (relg && i < n && relg[i] != (uint8_t)relv) return;
  uint64_t b = 0;
  if (i < n) {
    b = t[i];
    if (mark && l == 0) mark[i] = (uint8_t)markv;
    for (int64_t k = rp[i] + l; k < rp[i + 1]; k += 8)
      if (strong[k]) {
        const int32_t j = ci[k];
        const uint64_t tj = t[j];
        b = tj > b ? tj : b;
        if (mark) mark[j] = (uint8_t)markv;
      }
  }
  for (int o = 1; o < 8; o <<= 1) {
    const uint64_t x = (uint64_t)__shfl_xor((long long)b, o, 8);
    b = x > b ? x : b;
  }
  if (i < n && l == 0) m[i] = b;
}

// undecided i: root when it is the maximum of its neighbourhood, out when a
// root is in it; counts the undecided that remain
__global__ void k_amg_mis_update(int64_t n, uint64_t* __restrict__ t, const uint64_t* __restrict__ m,
                                 unsigned long long* __restrict__ left)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool undecided = false;
  if (i < n) {
    const uint64_t ti = t[i];
    if ((ti >> 62) == 1) {
      const uint64_t mi = m[i];
      if (mi == ti)
        t[i] = (2ull << 62) | (ti & ((1ull << 62) - 1));
      else if ((mi >> 62) == 2)
        t[i] = ti & ((1ull << 62) - 1);  // out
      else
        undecided = true;
    }
  }
  // one count per workgroup (a thread's own atomic on the one address serialised
  // millions of them in the first rounds; one per wave still cost 0.2-0.7 ms a round)
  __shared__ unsigned int cnt;
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  const unsigned long long w = __ballot(undecided);
  if ((threadIdx.x & 63) == 0 && w) atomicAdd(&cnt, (unsigned int)__popcll(w));
  __syncthreads();
  if (threadIdx.x == 0 && cnt) atomicAdd(left, (unsigned long long)cnt);
}

__global__ void k_amg_root_flags(int64_t n, const uint64_t* __restrict__ t, int32_t* __restrict__ f)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  f[i] = (t[i] >> 62) == 2 ? 1 : 0;
}

// roots: their aggregate (rank among the roots); others -1
__global__ void k_amg_root_agg(int64_t n, const uint64_t* __restrict__ t, const int64_t* __restrict__ rank,
                               int32_t* __restrict__ agg, uint64_t* __restrict__ owner)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool root = (t[i] >> 62) == 2;
  agg[i] = root ? (int32_t)rank[i] : -1;
  owner[i] = root ? t[i] : 0ull;  // the tuple of the node's root (0: none yet)
}

// unassigned graph nodes join the strong neighbour whose root tuple is the
// largest among the neighbours assigned in the previous pass (pass 1: roots).
// 8 lanes per row (its columns read coalesced), the largest tuple by a butterfly
// over the lanes: root tuples are unique per root, so equal tuples carry the same
// aggregate and the result is the row-order scan's
__global__ __launch_bounds__(256) void k_amg_join(int64_t n, const int64_t* __restrict__ rp,
                                                  const int32_t* __restrict__ ci, const uint8_t* __restrict__ strong,
                                                  const uint8_t* __restrict__ in, const int32_t* __restrict__ agg_in,
                                                  const uint64_t* __restrict__ own_in, int32_t* __restrict__ agg_out,
                                                  uint64_t* __restrict__ own_out)
{
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3;
  const int l = threadIdx.x & 7;
  int32_t a = -1;
  uint64_t o = 0;
  if (i < n) {
    a = agg_in[i];
    o = own_in[i];
    if (a < 0 && in[i]) {
      for (int64_t k = rp[i] + l; k < rp[i + 1]; k += 8) {
        const int32_t j = ci[k];
        if (!strong[k]) continue;
        const int32_t aj = agg_in[j];
        if (aj < 0) continue;
        const uint64_t oj = own_in[j];
        if (oj > o) {
          o = oj;
          a = aj;
        }
      }
    }
  }
  for (int w = 1; w < 8; w <<= 1) {
    const uint64_t ox = (uint64_t)__shfl_xor((long long)o, w, 8);
    const int32_t ax = __shfl_xor(a, w, 8);
    if (ox > o) {
      o = ox;
      a = ax;
    }
  }
  if (i < n && l == 0) {
    agg_out[i] = a;
    own_out[i] = o;
  }
}

// graph nodes no root reaches (isolated, or distance > hops): flag, to become
// singleton aggregates
__global__ void k_amg_orphans(int64_t n, const uint8_t* __restrict__ in, const int32_t* __restrict__ agg,
                              int32_t* __restrict__ f)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  f[i] = (in[i] && agg[i] < 0) ? 1 : 0;
}

__global__ void k_amg_orphan_agg(int64_t n, const int32_t* __restrict__ f, const int64_t* __restrict__ rank,
                                 int32_t base, int32_t* __restrict__ agg)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (f[i]) agg[i] = base + (int32_t)rank[i];
}

// run heads of the sorted keys (valid keys only)
__global__ void k_amg_heads(int64_t m, const unsigned long long* __restrict__ key, int32_t* __restrict__ head)
{
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= m) return;
  head[k] = key[k] != ~0ull && (k == 0 || key[k] != key[k - 1]) ? 1 : 0;
}

// the start of every run (heads scattered to their rank)
__global__ void k_amg_run_starts(int64_t m, const int32_t* __restrict__ head, const int64_t* __restrict__ hrank,
                                 int64_t* __restrict__ start)
{
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < m && head[k]) start[hrank[k]] = k;
}

// run r = [start r, start r+1): one thread per run, its sum in the sorted (=
// CSR) order (a thread per key whose heads looped over their runs left ~60 of
// 64 lanes idle: 10 ms at 172 M keys, r06aq)
__global__ void k_amg_runs(int64_t n_runs, int64_t m, const unsigned long long* __restrict__ key,
                           const double* __restrict__ vs, const int64_t* __restrict__ start, int64_t row_base,
                           int cbits, int64_t* __restrict__ c_row_of, int32_t* __restrict__ c_col,
                           double* __restrict__ c_val)
{
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_runs) return;
  const int64_t k0 = start[r];
  const unsigned long long kk = key[k0];
  double s = 0.0;
  for (int64_t q = k0; q < m && key[q] == kk; ++q) s += vs[q];
  c_row_of[r] = (int64_t)(kk >> cbits) - row_base;
  c_col[r] = (int32_t)(kk & ((1ull << cbits) - 1));
  c_val[r] = s;
}

// CSR row pointer of the coarse non-zeros (sorted by row)
__global__ void k_amg_rowptr(int64_t nnz, const int64_t* __restrict__ row_of, int64_t nc, int64_t* __restrict__ rp)
{
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nnz) return;
  const int64_t r = row_of[k];
  const int64_t prev = k > 0 ? row_of[k - 1] : -1;
  for (int64_t s = prev + 1; s <= r; ++s) rp[s] = k;
  if (k == nnz - 1)
    for (int64_t s = r + 1; s <= nc; ++s) rp[s] = nnz;
}

// aggregate member lists: members of aggregate a are mem[ap[a] .. ap[a+1]) in
// increasing fine index (stable sort of (agg, i))
__global__ void k_amg_member_keys(int64_t n, const int32_t* __restrict__ agg, uint32_t* __restrict__ key,
                                  int32_t* __restrict__ idx)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  key[i] = agg[i] >= 0 ? (uint32_t)agg[i] : 0xffffffffu;
  idx[i] = (int32_t)i;
}

__global__ void k_amg_member_ptr(int64_t n, const uint32_t* __restrict__ key, int64_t nc, int64_t* __restrict__ ap)
{
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int64_t a = key[k] == 0xffffffffu ? nc : (int64_t)key[k];
  const int64_t prev = k > 0 ? (key[k - 1] == 0xffffffffu ? nc : (int64_t)key[k - 1]) : -1;
  for (int64_t s = prev + 1; s <= a && s <= nc; ++s) ap[s] = k;
  if (k == n - 1)
    for (int64_t s = a + 1; s <= nc; ++s) ap[s] = n;
}

// y = A x (EPI 0), y = x + omega dinv (b - A x) (EPI 1), y = b - A x (EPI 2);
// 8 lanes per row, the row's products summed in a fixed butterfly order.  A
// lane's entries k, k + 8, ... four at a time: their columns and values, then
// the gathers, all in flight together (the sum in the same order as one entry
// at a time, bit for bit).  VT float: a level's fp32 copy of its values
// (AFEM_AMG_F32 = 2, the coarse levels)
template <int EPI, typename VT>
__global__ __launch_bounds__(256) void k_amg_spmv(int64_t n, const int64_t* __restrict__ rp,
                                                  const int32_t* __restrict__ ci, const VT* __restrict__ v,
                                                  const double* __restrict__ x, double* __restrict__ y,
                                                  const double* __restrict__ b, const double* __restrict__ dinv,
                                                  double omega)
{
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3;
  const int l = threadIdx.x & 7;
  double s = 0.0;
  if (i < n) {
    const int64_t k1 = rp[i + 1];
    for (int64_t kb = rp[i] + l; kb < k1; kb += 32) {
      int32_t c[4];
      VT w[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t k = kb + 8 * u;
        c[u] = k < k1 ? ci[k] : 0;
        w[u] = k < k1 ? v[k] : VT(0);
      }
      double xv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) xv[u] = x[c[u]];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (kb + 8 * u < k1) s += (double)w[u] * xv[u];
    }
  }
  s += __shfl_xor(s, 1, 8);
  s += __shfl_xor(s, 2, 8);
  s += __shfl_xor(s, 4, 8);
  if (i < n && l == 0) {
    if (EPI == 0) y[i] = s;
    if (EPI == 1) y[i] = x[i] + omega * dinv[i] * (b[i] - s);
    if (EPI == 2) y[i] = b[i] - s;
  }
}

// the fine level's epilogues after the PCG's own SpMV (q = A x):
// r = b - q, and x += omega dinv (b - q)
__global__ void k_amg_resid(int64_t n, const double* __restrict__ b, const double* __restrict__ q,
                            double* __restrict__ r)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    r[i] = b[i] - q[i];
}

__global__ void k_amg_jacobi(int64_t n, double omega, const double* __restrict__ dinv, const double* __restrict__ b,
                             const double* __restrict__ q, double* __restrict__ x)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] += omega * dinv[i] * (b[i] - q[i]);
}

__global__ void k_amg_scale(int64_t n, double omega, const double* __restrict__ dinv, const double* __restrict__ b,
                            double* __restrict__ x)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] = omega * dinv[i] * b[i];
}

// the fine level's cycle products on an fp32 copy of its values (AFEM_AMG_F32):
// CSR-stream over 256-row blocks (the block's value / column segment read with
// 16-B loads, four groups of 4 per lane in flight, products to LDS in a rotated
// order, one lane per row sums its products in CSR order) with the cycle's
// epilogue fused: EPI 2 y = b - A x (the residual), EPI 1 y = x + omega dinv
// (b - A x) (a Jacobi sweep; y must not be x), EPI 3 the sweep written into the
// preconditioner's output with its constraint rows (rin dfix: amg_apply's copy
// and k_amg_fix folded in).  The values are the preconditioner's
// only: the PCG's own product stays in fp64.  8 instead of 12 B per non-zero
__global__ void k_amg_d2f(int64_t n, const double* __restrict__ v, float* __restrict__ f)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    f[i] = (float)fmin(fmax(v[i], -3.4028234663852886e38), 3.4028234663852886e38);  // (a penalty beyond fp32: its
                                                                                      // largest value, never inf)
}

__global__ __launch_bounds__(256) void k_amg_seg256(int64_t n_rows, const int64_t* __restrict__ rp,
                                                    unsigned long long* __restrict__ mx)
{
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r0 = b * 256;
  if (r0 >= n_rows) return;
  const int64_t r1 = r0 + 256 < n_rows ? r0 + 256 : n_rows;
  atomicMax(mx, (unsigned long long)(rp[r1] - rp[r0]));
}

template <int EPI>
__global__ __launch_bounds__(256) void k_amg_f32(int64_t n_rows, int64_t nnz, const int64_t* __restrict__ rp,
                                                 const int32_t* __restrict__ ci, const float* __restrict__ vf,
                                                 const double* __restrict__ x, const double* __restrict__ b,
                                                 const double* __restrict__ dinv, double omega,
                                                 double* __restrict__ y, const uint8_t* __restrict__ cons = nullptr,
                                                 const double* __restrict__ rin = nullptr,
                                                 const double* __restrict__ dfix = nullptr)
{
  constexpr int U = 4;
  extern __shared__ __align__(16) unsigned char smem[];
  double* prod = reinterpret_cast<double*>(smem);
  const int64_t q8 = gridDim.x >> 3, rem = gridDim.x & 7;
  const int64_t xcd = blockIdx.x & 7;
  const int64_t blk = xcd * q8 + (xcd < rem ? xcd : rem) + (blockIdx.x >> 3);  // each XCD a contiguous range
  const int64_t r0 = blk * 256;
  const int64_t r1 = r0 + 256 < n_rows ? r0 + 256 : n_rows;
  const int64_t a = rp[r0], e = rp[r1];
  const int64_t q0 = (a & ~int64_t(3)) + 4 * (int64_t)threadIdx.x;
  auto load4 = [&](int64_t q, int (&c)[4], double (&v)[4]) {
    if (q + 4 <= nnz) {
      const int4 c4 = *reinterpret_cast<const int4*>(ci + q);
      const float4 f4 = *reinterpret_cast<const float4*>(vf + q);
      c[0] = c4.x;
      c[1] = c4.y;
      c[2] = c4.z;
      c[3] = c4.w;
      v[0] = f4.x;
      v[1] = f4.y;
      v[2] = f4.z;
      v[3] = f4.w;
    }
    else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        c[j] = q + j < nnz ? ci[q + j] : 0;
        v[j] = q + j < nnz ? (double)vf[q + j] : 0.0;
      }
    }
  };
  const int rot = (int)(threadIdx.x >> 3) & 3;
  auto put4 = [&](int64_t q, const double (&v)[4], const double (&xv)[4]) {
    double pr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) pr[j] = v[j] * xv[j];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int j = (t + rot) & 3;
      const double w = j == 0 ? pr[0] : (j == 1 ? pr[1] : (j == 2 ? pr[2] : pr[3]));
      if (q + j >= a && q + j < e) prod[q + j - a] = w;
    }
  };
  {
    int c[U][4];
    double v[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t q = q0 + (int64_t)u * 1024;
      if (q < e) {
        load4(q, c[u], v[u]);
      }
      else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          c[u][j] = 0;
          v[u][j] = 0.0;
        }
      }
    }
    double xv[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) xv[u][j] = x[c[u][j]];
#pragma unroll
    for (int u = 0; u < U; ++u) put4(q0 + (int64_t)u * 1024, v[u], xv[u]);
  }
  for (int64_t q = q0 + (int64_t)U * 1024; q < e; q += 1024) {
    int c[4];
    double v[4];
    load4(q, c, v);
    double xv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) xv[j] = x[c[j]];
    put4(q, v, xv);
  }
  __syncthreads();
  const int64_t r = r0 + threadIdx.x;
  if (r < r1) {
    double s = 0.0;
    for (int64_t k = rp[r] - a, kend = rp[r + 1] - a; k < kend; ++k) s += prod[k];
    if (EPI == 0)
      y[r] = s;
    else if (EPI == 2)
      y[r] = b[r] - s;
    else if (EPI == 3)
      y[r] = cons[r] ? rin[r] * dfix[r] : x[r] + omega * dinv[r] * (b[r] - s);
    else
      y[r] = x[r] + omega * dinv[r] * (b[r] - s);
  }
}

__global__ void k_amg_inv(int64_t n, const double* __restrict__ diag, const uint8_t* __restrict__ in,
                          double* __restrict__ dinv)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dinv[i] = in[i] ? 1.0 / diag[i] : 0.0;
}

// b_c[a] = sum of the members' r, in member order
__global__ void k_amg_restrict(int64_t nc, const int64_t* __restrict__ ap, const int32_t* __restrict__ mem,
                               const double* __restrict__ r, double* __restrict__ bc)
{
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= nc) return;
  // the members 16 at a time: their indices, then their values, all in flight
  // together, summed in member order (the serial loop's sum, bit for bit; it
  // waited on two dependent loads per member: 210 us per level-0 restriction at
  // 11.5 M rows, r06y)
  double s = 0.0;
  const int64_t q0 = ap[a], q1 = ap[a + 1];
  for (int64_t qb = q0; qb < q1; qb += 16) {
    int32_t mi[16];
    double rv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) mi[u] = qb + u < q1 ? mem[qb + u] : -1;
#pragma unroll
    for (int u = 0; u < 16; ++u) rv[u] = mi[u] >= 0 ? r[mi[u]] : 0.0;
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (qb + u < q1) s += rv[u];
  }
  bc[a] = s;
}

__global__ void k_amg_prolong(int64_t n, const int32_t* __restrict__ agg, double scale, const double* __restrict__ xc,
                              double* __restrict__ x)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (agg[i] >= 0) x[i] += scale * xc[agg[i]];
}

__global__ void k_amg_mask(int64_t n, const uint8_t* __restrict__ cons, const double* __restrict__ r,
                           double* __restrict__ b)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    b[i] = cons[i] ? 0.0 : r[i];
}

// b = F r and the first sweep from zero x = omega dinv b in one pass (amg_apply's entry)
__global__ void k_amg_mask_scale(int64_t n, const uint8_t* __restrict__ cons, const double* __restrict__ r,
                                 double omega, const double* __restrict__ dinv, double* __restrict__ b,
                                 double* __restrict__ x)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double bi = cons[i] ? 0.0 : r[i];
    b[i] = bi;
    x[i] = omega * dinv[i] * bi;
  }
}

__global__ void k_amg_fix(int64_t n, const uint8_t* __restrict__ cons, const double* __restrict__ r,
                          const double* __restrict__ dinv, double* __restrict__ z)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (cons[i]) z[i] = r[i] * dinv[i];
}

__global__ void k_amg_fill(int64_t n, const uint8_t* __restrict__ in, double* __restrict__ v)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    v[i] = in[i] ? (double)(h & 0xFFFF) / 32768.0 - 1.0 : 0.0;  // signed: every mode gets a share
  }
}

// w = dinv .* w, block partials of w.w (and of v.v when v is given)
__global__ void k_amg_dscale_dot(int64_t n, const double* __restrict__ dinv, double* __restrict__ w,
                                 double* __restrict__ partial)
{
  __shared__ double sh[256];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double t = dinv ? dinv[i] * w[i] : w[i];
    w[i] = t;
    s += t * t;
  }
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = sh[0];
}

__global__ void k_amg_mul(int64_t n, double a, double* __restrict__ v)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    v[i] *= a;
}

// power iteration on the device (one rank): st = {norm of the previous iterate,
// lambda, 1 / norm of this one, stopped}.  The partials summed in order by one
// thread (the host loop's sum, bit for bit); first = the initial vector's norm
__global__ void k_amg_pw_norm(const double* __restrict__ partial, int g, int first, double* __restrict__ st)
{
  if (threadIdx.x != 0 || st[3] != 0.0) return;
  double s = 0.0;
  int k = 0;
  for (; k + 8 <= g; k += 8) {  // the loads in flight together, the adds in order
    double p[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) p[u] = partial[k + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += p[u];
  }
  for (; k < g; ++k) s += partial[k];
  const double nw = sqrt(s);
  if (first) {
    st[0] = nw;
    return;
  }
  st[1] = st[0] > 0 ? nw / st[0] : 0.0;
  if (!(nw > 0)) {
    st[3] = 1.0;
    return;
  }
  st[2] = 1.0 / nw;
  st[0] = 1.0;
}

__global__ void k_amg_mul_dev(int64_t n, const double* __restrict__ st, double* __restrict__ v)
{
  if (st[3] != 0.0) return;
  const double a = st[2];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    v[i] *= a;
}

__global__ __launch_bounds__(64) void k_amg_gemv(int n, const double* __restrict__ A, const double* __restrict__ b,
                                                 double* __restrict__ x)
{
  const int i = blockIdx.x;
  double s = 0.0;
  for (int j = threadIdx.x; j < n; j += 64) s += A[(int64_t)i * n + j] * b[j];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (threadIdx.x == 0) x[i] = s;
}

// an independent set that did not settle: its undecided nodes become roots
// (aggregates may then touch; the aggregation stays valid)
__global__ void k_amg_promote(int64_t n, uint64_t* __restrict__ t)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t ti = t[i];
  if ((ti >> 62) == 1) t[i] = (2ull << 62) | (ti & ((1ull << 62) - 1));
}

// Galerkin keys through a column map: (row_base + agg i, cmap[j]) -- cmap is
// agg on one rank, the coarse local index (owned aggregates, then the coarse
// ghosts) on a distributed level, the global coarse index toward a gathered
// level; all ones outside the graph
__global__ void k_amg_keys_map(int64_t n, const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
                               const int32_t* __restrict__ agg, int64_t row_base, const int32_t* __restrict__ cmap,
                               int64_t ncol, int cbits, unsigned long long* __restrict__ key)
{
  // 8 lanes per row (the row's columns read and its keys written coalesced)
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3;
  if (i >= n) return;
  const int32_t ai = agg[i];
  for (int64_t k = rp[i] + (threadIdx.x & 7); k < rp[i + 1]; k += 8) {
    const int32_t j = ci[k];
    const int32_t aj = (j >= 0 && j < ncol) ? cmap[j] : -1;
    key[k] = (ai >= 0 && aj >= 0) ? ((unsigned long long)(row_base + ai) << cbits | (uint32_t)aj) : ~0ull;
  }
}

__global__ void k_amg_i2d(int64_t n, const int32_t* __restrict__ a, double* __restrict__ d)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) d[i] = (double)a[i];
}

// the gathered level's global COO (all-reduced as doubles) -> row ids, columns
__global__ void k_amg_coo_unpack(int64_t m, const double* __restrict__ r, const double* __restrict__ c,
                                 int64_t* __restrict__ row_of, int32_t* __restrict__ col)
{
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= m) return;
  row_of[k] = (int64_t)r[k];
  col[k] = (int32_t)c[k];
}

double env_double(const char* name, double dflt)
{
  const char* v = variant(name);
  return v && *v ? std::atof(v) : dflt;
}

}  // namespace

struct AmgLevel {
  int64_t n = 0, nnz = 0;
  // columns of the level's vectors: n on one rank and on replicated levels;
  // owned + ghost columns on a distributed level (the ghost part filled by
  // the level's halo exchange before every product)
  int64_t ncol = 0;
  bool dist = false;
  Halo* H = nullptr;               // the level's halo (level 0: the system's; coarser: own_halo)
  std::unique_ptr<Halo> own_halo;
  // the next level replicated on every rank (gathered): this rank's
  // aggregates are its rows [gather_off, gather_off + nc_local)
  int64_t gather_off = -1, nc_local = 0;
  // a distributed level small enough to be solved whole: gathered as it is
  // (identity aggregates) onto the next level, its cycle = gather b, solve
  // there, take back this rank's part (no smoothing here)
  bool pass = false;
  const int64_t* rp = nullptr;
  const int32_t* ci = nullptr;
  const double* v = nullptr;
  DevBuf<int64_t> own_rp;
  DevBuf<int32_t> own_ci;
  DevBuf<double> own_v;
  DevBuf<double> diag, dinv;
  DevBuf<uint8_t> in;        // row in the strength graph
  DevBuf<int32_t> agg;       // row -> aggregate of the next level, -1 outside
  DevBuf<int64_t> ap;        // aggregate members (next level's rows): CSR over the fine rows
  DevBuf<int32_t> mem;
  DevBuf<double> x, t, b, r;
  DevBuf<double> kc1, kv1, krt, kcoef;  // K-cycle level (Amg::kcycle)
  DevBuf<float> v32;                    // AFEM_AMG_F32 = 2: a coarse level's values in fp32 (its cycle products)
  double omega = 0.0;
};

struct Amg {
  std::vector<AmgLevel> lv;
  DevBuf<double> ainv;
  int n_dense = 0;
  int sweeps = 1;
  double scale = 1.0;
  // AFEM_AMG_POWER_ITS: power iterations per level for lambda_max (kPowerIts)
  int power_its = kPowerIts;
  double omega_scale = 1.0;  // AFEM_AMG_OMEGA: a factor on every level's omega (measurements)
  // AFEM_AMG_KCYCLE=k: levels 1..k solve their coarse problem by two flexible-CG
  // steps preconditioned by the cycle below (K-cycle) instead of one cycle
  int kcycle = 0;
  bool fine_planned = true;
  // AFEM_AMG_F32 (one rank): the fine level's cycle products on an fp32 copy of
  // its values (k_amg_f32, epilogues fused); f32_seg: the largest 256-row segment
  DevBuf<float> v32;
  int64_t f32_seg = 0;
  // several ranks: the communicator of the distributed levels (null on one rank)
  Comm* comm = nullptr;
  DevBuf<double> sums;  // all-reduced scalars (power iterations, K-cycle steps)
  // AFEM_AMG_GRAPH=1: the V-cycle replayed as a captured HIP graph (its
  // launches are fixed once the hierarchy is); keyed on (r, z, the solve's
  // SpMV plan).  Measured equal (2.93 ms per iteration either way, r05aa):
  // the cycle is bound by its three fine-level products, not by launches.
  // One rank only (a distributed cycle exchanges halos through the transport)
  bool use_graph = true;
  hipGraphExec_t gexec = nullptr;
  const double* g_r = nullptr;
  double* g_z = nullptr;
  const void* g_plan = nullptr;  // the solve's SpMV plan the graph's fine products were captured with
  ~Amg()
  {
    if (gexec) (void)hipGraphExecDestroy(gexec);
  }
  DevBuf<double> partial;
  const void* key_rows = nullptr;
  const void* key_cols = nullptr;
  const void* key_vals = nullptr;
  int64_t key_n = 0, key_nnz = 0;
};

void AmgDeleter::operator()(Amg* a) const { delete a; }

namespace {
bool multi_rank(const LinearSystem& ls)
{
  return ls.halo && ls.halo->comm && (comm_nranks(ls.halo->comm) > 1 || comm_self_loop());
}
}  // namespace

bool amg_available(const LinearSystem& ls)
{
  // (several ranks: a rank without rows still takes part -- every rank must
  // make the same choice, or the collectives of the setup and the cycle mismatch)
  if (!ls.csr_rows || !ls.csr_cols || !ls.csr_vals || (ls.n_rows <= 0 && !multi_rank(ls))) return false;
  if (multi_rank(ls) && ls.n_cols < ls.n_rows) return false;
  // hipcub's sorts of the setup take int counts: the non-zeros of every level
  // (the fine level's are the most) must stay below 2^31, else point Jacobi
  return ls.n_rows < (int64_t(1) << 31) && ls.csr_nnz < (int64_t(1) << 31);
}

bool amg_nonlinear(const LinearSystem& ls)
{
  if (!ls.amg) return false;
  for (const auto& L : ls.amg->lv)
    if (L.kcoef.p) return true;
  return false;
}

int amg_levels(const LinearSystem& ls) { return ls.amg ? (int)ls.amg->lv.size() : 0; }

namespace {

double host_sum(Ctx& ctx, const DevBuf<double>& partial, int n)
{
  std::vector<double> h(n);
  AFEM_HIP(hipMemcpyAsync(h.data(), partial.p, n * sizeof(double), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  double s = 0.0;
  for (double v : h) s += v;
  return s;
}

// the sum of v over the ranks (v itself on one rank)
double allsum(Ctx& ctx, Amg& a, double v)
{
  if (!a.comm) return v;
  AFEM_HIP(hipMemcpyAsync(a.sums.p, &v, sizeof(double), hipMemcpyHostToDevice, ctx.stream));
  comm_allreduce(a.comm, ctx, a.sums.p, 1);
  double r = 0.0;
  AFEM_HIP(hipMemcpyAsync(&r, a.sums.p, sizeof(double), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  return r;
}

// element-wise sums over the ranks of a host vector
std::vector<double> allsum_vec(Ctx& ctx, Amg& a, std::vector<double> h)
{
  if (!a.comm || h.empty()) return h;
  DevBuf<double> d;
  d.alloc(h.size());
  AFEM_HIP(hipMemcpyAsync(d.p, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice, ctx.stream));
  comm_allreduce(a.comm, ctx, d.p, (int64_t)h.size());
  AFEM_HIP(hipMemcpyAsync(h.data(), d.p, h.size() * sizeof(double), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  return h;
}

void spmv(Ctx& ctx, int epi, AmgLevel& L, const double* x, double* y, const double* b, double omega,
          bool exact = false)
{
  const unsigned g = grid_for(L.n * 8, 256);
  if (L.n == 0) return;
  // exact: the products that must be the level's operator itself (power iteration, K-cycle Krylov steps)
  const float* vf = exact ? nullptr : L.v32.p;
#define AFEM_AMG_SPMV(E)                                                                                         \
  if (vf)                                                                                                        \
    hipLaunchKernelGGL((k_amg_spmv<E, float>), dim3(g), dim3(256), 0, ctx.stream, L.n, L.rp, L.ci, vf, x, y, b,   \
                       L.dinv.p, omega);                                                                          \
  else                                                                                                           \
    hipLaunchKernelGGL((k_amg_spmv<E, double>), dim3(g), dim3(256), 0, ctx.stream, L.n, L.rp, L.ci, L.v, x, y, b, \
                       L.dinv.p, omega);
  if (epi == 0) {
    AFEM_AMG_SPMV(0)
  }
  else if (epi == 1) {
    AFEM_AMG_SPMV(1)
  }
  else {
    AFEM_AMG_SPMV(2)
  }
#undef AFEM_AMG_SPMV
  AFEM_LAUNCHED();
}

// the ghost part of a distributed level's vector (nothing on other levels)
void halo(Ctx& ctx, AmgLevel& L, double* x)
{
  if (L.dist && L.H) halo_exchange(*L.H, ctx, x);
}

// the fine level's cycle product on the fp32 values with its epilogue (k_amg_f32)
void f32_product(Ctx& ctx, Amg& a, AmgLevel& L, int epi, const double* x, const double* b, double* y,
                 const uint8_t* cons = nullptr, const double* rin = nullptr, const double* dfix = nullptr)
{
  if (L.n == 0) return;
  const unsigned nb = (unsigned)((L.n + 255) / 256);
  const size_t shm = (size_t)a.f32_seg * 8 + 32;
  if (epi == 3)
    hipLaunchKernelGGL(k_amg_f32<3>, dim3(nb), dim3(256), shm, ctx.stream, L.n, L.nnz, L.rp, L.ci,
                       (const float*)a.v32.p, x, b, (const double*)L.dinv.p, L.omega, y, cons, rin, dfix);
  else if (epi == 0)
    hipLaunchKernelGGL(k_amg_f32<0>, dim3(nb), dim3(256), shm, ctx.stream, L.n, L.nnz, L.rp, L.ci,
                       (const float*)a.v32.p, x, b, (const double*)L.dinv.p, L.omega, y);
  else if (epi == 2)
    hipLaunchKernelGGL(k_amg_f32<2>, dim3(nb), dim3(256), shm, ctx.stream, L.n, L.nnz, L.rp, L.ci,
                       (const float*)a.v32.p, x, b, (const double*)L.dinv.p, L.omega, y);
  else
    hipLaunchKernelGGL(k_amg_f32<1>, dim3(nb), dim3(256), shm, ctx.stream, L.n, L.nnz, L.rp, L.ci,
                       (const float*)a.v32.p, x, b, (const double*)L.dinv.p, L.omega, y);
  AFEM_LAUNCHED();
}

// the fp32 copy of the fine level's values (setup, and every reuse of a kept hierarchy)
void f32_refresh(Ctx& ctx, Amg& a, const AmgLevel& L)
{
  if (!a.v32.p || L.nnz == 0) return;
  hipLaunchKernelGGL(k_amg_d2f, dim3((unsigned)std::min<int64_t>(kVec, (L.nnz + 255) / 256)), dim3(256), 0,
                     ctx.stream, L.nnz, L.v, a.v32.p);
  AFEM_LAUNCHED();
}

double power_lambda(Ctx& ctx, Amg& a, AmgLevel& L)
{
  const unsigned g = (unsigned)std::min<int64_t>(kVec, std::max<int64_t>(1, (L.n + 255) / 256));
  if (L.n > 0) {
    hipLaunchKernelGGL(k_amg_fill, dim3(g), dim3(256), 0, ctx.stream, L.n, L.in.p, L.x.p);
    hipLaunchKernelGGL(k_amg_dscale_dot, dim3(g), dim3(256), 0, ctx.stream, L.n, (const double*)nullptr, L.x.p,
                       a.partial.p);
    AFEM_LAUNCHED();
  }
  const bool d = L.dist;
  if (!d && L.n > 0) {
    // one rank: no host round trip per iteration (the same arithmetic and order)
    DevBuf<double> st;
    st.alloc(4);
    AFEM_HIP(hipMemsetAsync(st.p, 0, st.bytes(), ctx.stream));
    hipLaunchKernelGGL(k_amg_pw_norm, dim3(1), dim3(64), 0, ctx.stream, (const double*)a.partial.p, (int)g, 1, st.p);
    // (the fine level's products on its fp32 copy when it has one: lambda_max of the fp32-rounded
    // operator, the one the cycle's sweeps apply)
    const bool f32 = a.v32.p && &L == &a.lv[0];
    for (int it = 0; it < a.power_its; ++it) {
      if (f32)
        f32_product(ctx, a, L, 0, L.x.p, nullptr, L.t.p);
      else
        spmv(ctx, 0, L, L.x.p, L.t.p, nullptr, 0.0);
      hipLaunchKernelGGL(k_amg_dscale_dot, dim3(g), dim3(256), 0, ctx.stream, L.n, (const double*)L.dinv.p, L.t.p,
                         a.partial.p);
      hipLaunchKernelGGL(k_amg_pw_norm, dim3(1), dim3(64), 0, ctx.stream, (const double*)a.partial.p, (int)g, 0, st.p);
      hipLaunchKernelGGL(k_amg_mul_dev, dim3(g), dim3(256), 0, ctx.stream, L.n, (const double*)st.p, L.t.p);
      AFEM_LAUNCHED();
      std::swap(L.x, L.t);
    }
    double lam = 0.0;
    AFEM_HIP(hipMemcpyAsync(&lam, st.p + 1, sizeof(double), hipMemcpyDeviceToHost, ctx.stream));
    ctx.sync();
    return lam;
  }
  double nv = std::sqrt(d ? allsum(ctx, a, L.n > 0 ? host_sum(ctx, a.partial, (int)g) : 0.0)
                          : host_sum(ctx, a.partial, (int)g)),
         lam = 0.0;
  for (int it = 0; it < a.power_its; ++it) {
    halo(ctx, L, L.x.p);
    spmv(ctx, 0, L, L.x.p, L.t.p, nullptr, 0.0);
    if (L.n > 0) {
      hipLaunchKernelGGL(k_amg_dscale_dot, dim3(g), dim3(256), 0, ctx.stream, L.n, (const double*)L.dinv.p, L.t.p,
                         a.partial.p);
      AFEM_LAUNCHED();
    }
    const double ls = L.n > 0 ? host_sum(ctx, a.partial, (int)g) : 0.0;
    const double nw = std::sqrt(d ? allsum(ctx, a, ls) : ls);
    lam = nv > 0 ? nw / nv : 0.0;
    if (!(nw > 0)) break;
    if (L.n > 0) {
      hipLaunchKernelGGL(k_amg_mul, dim3(g), dim3(256), 0, ctx.stream, L.n, 1.0 / nw, L.t.p);
      AFEM_LAUNCHED();
    }
    std::swap(L.x, L.t);
    nv = 1.0;
  }
  return lam;
}

// the level's diagonal, graph membership, D^-1 and work vectors (x, t, r over
// the level's columns, zeroed: their ghost part is only ever written by the
// halo exchange)
void level_prepare(Ctx& ctx, AmgLevel& L, const uint8_t* cons)
{
  if (L.ncol < L.n) L.ncol = L.n;
  L.diag.alloc(L.n > 0 ? L.n : 1);
  L.in.alloc(L.n > 0 ? L.n : 1);
  L.dinv.alloc(L.n > 0 ? L.n : 1);
  for (auto* b : { &L.x, &L.t, &L.r }) {
    b->alloc(L.ncol > 0 ? L.ncol : 1);
    AFEM_HIP(hipMemsetAsync(b->p, 0, b->bytes(), ctx.stream));
  }
  L.b.alloc(L.n > 0 ? L.n : 1);
  if (L.n == 0) return;
  hipLaunchKernelGGL(k_amg_diag, dim3(grid_for(L.n, 256)), dim3(256), 0, ctx.stream, L.n, L.rp, L.ci, L.v, cons,
                     L.diag.p, L.in.p);
  const unsigned g = (unsigned)std::min<int64_t>(kVec, (L.n + 255) / 256);
  hipLaunchKernelGGL(k_amg_inv, dim3(g), dim3(256), 0, ctx.stream, L.n, L.diag.p, L.in.p, L.dinv.p);
  AFEM_LAUNCHED();
}

// aggregates of level L's own rows (L.agg, L.ap / L.mem); returns the
// aggregate count.  Ghost columns are outside the strength graph
// (k_amg_strength: j < n): a distributed level aggregates within each rank
int64_t aggregate(Ctx& ctx, AmgLevel& L, double theta, int hops)
{
  const int64_t n = L.n;
  if (n == 0) {
    L.agg.alloc(1);
    L.mem.alloc(1);
    L.ap.alloc(1);
    AFEM_HIP(hipMemsetAsync(L.ap.p, 0, sizeof(int64_t), ctx.stream));
    ctx.sync();
    return 0;
  }
  const unsigned g = grid_for(n, 256);
  DevBuf<uint64_t> t, m;
  t.alloc(n);
  m.alloc(n);
  hipLaunchKernelGGL(k_amg_tuple_init, dim3(g), dim3(256), 0, ctx.stream, n, L.in.p, t.p);
  AFEM_LAUNCHED();
  DevBuf<unsigned long long> left;
  left.alloc(1);
  DevBuf<uint8_t> strong;
  strong.alloc(L.nnz > 0 ? L.nnz : 1);
  const unsigned g8 = grid_for(n * 8, 256);
  hipLaunchKernelGGL(k_amg_strength, dim3(g8), dim3(256), 0, ctx.stream, n, L.rp, L.ci, L.v, L.diag.p, L.in.p, theta,
                     strong.p);
  AFEM_LAUNCHED();
  DevBuf<uint64_t> m2;
  DevBuf<uint8_t> rel;
  if (hops > 1) {
    m2.alloc(n);
    rel.alloc(n);
    AFEM_HIP(hipMemsetAsync(rel.p, 0, n, ctx.stream));
  }
  const bool verbose_rounds = env_double("AFEM_AMG_VERBOSE", 0.0) > 1;
  auto t_round = std::chrono::steady_clock::now();
  for (int round = 0; round < 64; ++round) {
    // max over the distance-`hops` neighbourhood (hops 2: the first hop over the rows
    // the previous round marked, the second over the undecided rows)
    hipLaunchKernelGGL(k_amg_maxprop, dim3(g8), dim3(256), 0, ctx.stream, n, L.rp, L.ci, (const uint8_t*)strong.p,
                       (const uint64_t*)t.p, m.p, hops == 1 ? (const uint64_t*)t.p : nullptr,
                       hops > 1 && round > 0 ? (const uint8_t*)rel.p : nullptr, round, (uint8_t*)nullptr, 0);
    for (int h = 1; h < hops; ++h) {
      hipLaunchKernelGGL(k_amg_maxprop, dim3(g8), dim3(256), 0, ctx.stream, n, L.rp, L.ci, (const uint8_t*)strong.p,
                         (const uint64_t*)m.p, m2.p, h + 1 == hops ? (const uint64_t*)t.p : nullptr,
                         (const uint8_t*)nullptr, 0, h + 1 == hops ? rel.p : (uint8_t*)nullptr, round + 1);
      std::swap(m, m2);
    }
    AFEM_HIP(hipMemsetAsync(left.p, 0, sizeof(unsigned long long), ctx.stream));
    hipLaunchKernelGGL(k_amg_mis_update, dim3(g), dim3(256), 0, ctx.stream, n, t.p, (const uint64_t*)m.p, left.p);
    AFEM_LAUNCHED();
    unsigned long long hl = 0;
    AFEM_HIP(hipMemcpyAsync(&hl, left.p, sizeof(hl), hipMemcpyDeviceToHost, ctx.stream));
    ctx.sync();
    if (verbose_rounds) {  // AFEM_AMG_VERBOSE=2: each round's wall time and undecided rows
      const auto t = std::chrono::steady_clock::now();
      std::fprintf(stderr, "amg round %2d: %8.3f ms, %llu undecided\n", round,
                   std::chrono::duration<double, std::milli>(t - t_round).count(), hl);
      t_round = t;
    }
    if (hl == 0) {
      if (env_double("AFEM_AMG_VERBOSE", 0.0) > 0) std::fprintf(stderr, "amg: independent set in %d rounds\n", round + 1);
      break;
    }
    if (round == 63) {
      //  the independent set did not settle in 64 rounds: the
      // undecided nodes become roots instead of failing the solve
      hipLaunchKernelGGL(k_amg_promote, dim3(g), dim3(256), 0, ctx.stream, n, t.p);
      AFEM_LAUNCHED();
    }
  }
  auto t_tail = std::chrono::steady_clock::now();
  DevBuf<int32_t> f;
  DevBuf<int64_t> rank;
  f.alloc(n);
  rank.alloc(n + 1);
  hipLaunchKernelGGL(k_amg_root_flags, dim3(g), dim3(256), 0, ctx.stream, n, (const uint64_t*)t.p, f.p);
  AFEM_LAUNCHED();
  exclusive_scan_i32_to_i64(ctx, f.p, rank.p, n);
  const int64_t n_roots = read_i64(ctx, rank.p + n);
  L.agg.alloc(n);
  DevBuf<int32_t> agg2;
  DevBuf<uint64_t> own, own2;
  agg2.alloc(n);
  own.alloc(n);
  own2.alloc(n);
  hipLaunchKernelGGL(k_amg_root_agg, dim3(g), dim3(256), 0, ctx.stream, n, (const uint64_t*)t.p, rank.p, L.agg.p,
                     own.p);
  AFEM_LAUNCHED();
  for (int h = 0; h < hops; ++h) {
    hipLaunchKernelGGL(k_amg_join, dim3(grid_for(n * 8, 256)), dim3(256), 0, ctx.stream, n, L.rp, L.ci, (const uint8_t*)strong.p,
                       L.in.p, (const int32_t*)L.agg.p, (const uint64_t*)own.p, agg2.p, own2.p);
    AFEM_LAUNCHED();
    std::swap(L.agg, agg2);
    std::swap(own, own2);
  }
  // orphans (no root within reach) become singletons after the roots' aggregates
  hipLaunchKernelGGL(k_amg_orphans, dim3(g), dim3(256), 0, ctx.stream, n, L.in.p, L.agg.p, f.p);
  AFEM_LAUNCHED();
  exclusive_scan_i32_to_i64(ctx, f.p, rank.p, n);
  const int64_t n_orph = read_i64(ctx, rank.p + n);
  if (n_orph) {
    hipLaunchKernelGGL(k_amg_orphan_agg, dim3(g), dim3(256), 0, ctx.stream, n, f.p, rank.p, (int32_t)n_roots,
                       L.agg.p);
    AFEM_LAUNCHED();
  }
  const int64_t nc = n_roots + n_orph;
  // member lists
  DevBuf<uint32_t> k1, k2;
  DevBuf<int32_t> i1;
  k1.alloc(n);
  k2.alloc(n);
  i1.alloc(n);
  L.mem.alloc(n);
  hipLaunchKernelGGL(k_amg_member_keys, dim3(g), dim3(256), 0, ctx.stream, n, L.agg.p, k1.p, i1.p);
  AFEM_LAUNCHED();
  size_t tb = 0;
  AFEM_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k1.p, k2.p, i1.p, L.mem.p, (int)n, 0, 32, ctx.stream));
  DevBuf<unsigned char> tmp;
  tmp.alloc(tb > 0 ? tb : 1);
  AFEM_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, k1.p, k2.p, i1.p, L.mem.p, (int)n, 0, 32, ctx.stream));
  L.ap.alloc(nc + 1);
  AFEM_HIP(hipMemsetAsync(L.ap.p, 0, (nc + 1) * sizeof(int64_t), ctx.stream));
  hipLaunchKernelGGL(k_amg_member_ptr, dim3(g), dim3(256), 0, ctx.stream, n, (const uint32_t*)k2.p, nc, L.ap.p);
  AFEM_LAUNCHED();
  ctx.sync();
  if (verbose_rounds)
    std::fprintf(stderr, "amg aggregates from the set (joins, orphans, members): %8.3f ms\n",
                 std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_tail).count());
  return nc;
}

// The coarse operator's non-zeros of level L's rows, keyed (row_base + agg i,
// cmap[j]): radix-sorted (stable), each run summed in the CSR order.  Out: the
// rows (relative to row_base) of the n_out coarse rows, their columns and
// values (COO in row order) and their count.  row_bound / col_bound: exclusive
// bounds of row_base + agg i and of cmap[j]; the key packs them into
// bitlen(row_bound) + bitlen(col_bound - 1) bits and the sort runs over those
// only (5 digit passes instead of 8 at the unstructured leg's 11.5 M rows); the
// sort carries the values themselves (the runs then sum contiguous values: the
// gather through sorted source positions cost 16 ms at that size, r06y).  An
// invalid key (~0) is all ones in the sorted bits, which no valid key is
// (row < 2^rbits - 1).
int64_t galerkin_coo(Ctx& ctx, AmgLevel& L, const int32_t* cmap, int64_t ncol, int64_t row_base, int64_t row_bound,
                     int64_t col_bound, DevBuf<int64_t>& row_of, DevBuf<int32_t>& col, DevBuf<double>& val)
{
  const int64_t nnz = L.nnz;
  auto bitlen = [](uint64_t x) {
    int b = 0;
    while (x) {
      ++b;
      x >>= 1;
    }
    return b;
  };
  const int cbits = std::max(1, bitlen((uint64_t)std::max<int64_t>(col_bound - 1, 0)));
  const int rbits = bitlen((uint64_t)std::max<int64_t>(row_bound, 1));
  AFEM_REQUIRE(cbits <= 32 && cbits + rbits <= 64, AFEM_ERR_LIMIT, "amg: coarse key above 64 bits");
  DevBuf<unsigned long long> key, key_s;
  DevBuf<double> val_s;
  key.alloc(nnz > 0 ? nnz : 1);
  key_s.alloc(nnz > 0 ? nnz : 1);
  val_s.alloc(nnz > 0 ? nnz : 1);
  if (L.n > 0) {
    hipLaunchKernelGGL(k_amg_keys_map, dim3(grid_for(L.n * 8, 256)), dim3(256), 0, ctx.stream, L.n, L.rp, L.ci,
                       (const int32_t*)L.agg.p, row_base, cmap, ncol, cbits, key.p);
    AFEM_LAUNCHED();
  }
  size_t tb = 0;
  AFEM_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, key.p, key_s.p, L.v, val_s.p, (int)nnz, 0, cbits + rbits,
                                              ctx.stream));
  DevBuf<unsigned char> tmp;
  tmp.alloc(tb > 0 ? tb : 1);
  AFEM_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, key.p, key_s.p, L.v, val_s.p, (int)nnz, 0, cbits + rbits,
                                              ctx.stream));
  key.reset();
  tmp.reset();
  DevBuf<int32_t> head;
  DevBuf<int64_t> hrank;
  head.alloc(nnz > 0 ? nnz : 1);
  hrank.alloc(nnz + 1);
  if (nnz > 0) {
    hipLaunchKernelGGL(k_amg_heads, dim3(grid_for(nnz, 256)), dim3(256), 0, ctx.stream, nnz,
                       (const unsigned long long*)key_s.p, head.p);
    AFEM_LAUNCHED();
  }
  exclusive_scan_i32_to_i64(ctx, head.p, hrank.p, nnz);
  const int64_t cnnz = read_i64(ctx, hrank.p + nnz);
  row_of.alloc(cnnz > 0 ? cnnz : 1);
  col.alloc(cnnz > 0 ? cnnz : 1);
  val.alloc(cnnz > 0 ? cnnz : 1);
  if (nnz > 0 && cnnz > 0) {
    DevBuf<int64_t> start;
    start.alloc(cnnz);
    hipLaunchKernelGGL(k_amg_run_starts, dim3(grid_for(nnz, 256)), dim3(256), 0, ctx.stream, nnz, head.p, hrank.p,
                       start.p);
    hipLaunchKernelGGL(k_amg_runs, dim3(grid_for(cnnz, 256)), dim3(256), 0, ctx.stream, cnnz, nnz,
                       (const unsigned long long*)key_s.p, (const double*)val_s.p, (const int64_t*)start.p, row_base,
                       cbits, row_of.p, col.p, val.p);
    AFEM_LAUNCHED();
  }
  ctx.sync();
  return cnnz;
}

// C's CSR from its COO (rows sorted): C.own_rp / own_ci / own_v
void coo_to_level(Ctx& ctx, int64_t n_rows, int64_t cnnz, DevBuf<int64_t>& row_of, DevBuf<int32_t>& col,
                  DevBuf<double>& val, AmgLevel& C)
{
  C.own_rp.alloc(n_rows + 1);
  AFEM_HIP(hipMemsetAsync(C.own_rp.p, 0, (n_rows + 1) * sizeof(int64_t), ctx.stream));
  if (cnnz > 0) {
    hipLaunchKernelGGL(k_amg_rowptr, dim3(grid_for(cnnz, 256)), dim3(256), 0, ctx.stream, cnnz, row_of.p, n_rows,
                       C.own_rp.p);
    AFEM_LAUNCHED();
  }
  ctx.sync();
  C.own_ci = std::move(col);
  C.own_v = std::move(val);
  C.n = n_rows;
  C.nnz = cnnz;
  C.rp = C.own_rp.p;
  C.ci = C.own_ci.p;
  C.v = C.own_v.p;
}

// C = P^T A P of level L's aggregates on one rank (or a replicated level)
void galerkin(Ctx& ctx, AmgLevel& L, int64_t nc, AmgLevel& C)
{
  DevBuf<int64_t> row_of;
  DevBuf<int32_t> col;
  DevBuf<double> val;
  const int64_t cnnz = galerkin_coo(ctx, L, L.agg.p, L.n, 0, nc, nc, row_of, col, val);
  coo_to_level(ctx, nc, cnnz, row_of, col, val, C);
  C.ncol = nc;
}

// the host copy of a device int array
std::vector<int32_t> to_host_i32(Ctx& ctx, const int32_t* d, int64_t n)
{
  std::vector<int32_t> h(n);
  if (n) AFEM_HIP(hipMemcpyAsync(h.data(), d, n * sizeof(int32_t), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  return h;
}

// Level L (distributed) and its aggregates: for every ghost column, its
// owner's aggregate (the aggregate ids exchanged through L's halo as doubles)
// and its owner rank (the neighbour whose receive list holds it)
void ghost_aggregates(Ctx& ctx, AmgLevel& L, std::vector<int32_t>& gagg, std::vector<int32_t>& gown)
{
  const int64_t ng = L.ncol - L.n;
  DevBuf<double> gv;
  gv.alloc(L.ncol > 0 ? L.ncol : 1);
  AFEM_HIP(hipMemsetAsync(gv.p, 0, gv.bytes(), ctx.stream));
  if (L.n > 0) {
    hipLaunchKernelGGL(k_amg_i2d, dim3(grid_for(L.n, 256)), dim3(256), 0, ctx.stream, L.n, (const int32_t*)L.agg.p,
                       gv.p);
    AFEM_LAUNCHED();
  }
  halo_exchange(*L.H, ctx, gv.p);
  std::vector<double> h(ng);
  if (ng) AFEM_HIP(hipMemcpyAsync(h.data(), gv.p + L.n, ng * sizeof(double), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  gagg.assign(ng, -1);
  gown.assign(ng, -1);
  const Halo& H = *L.H;
  const std::vector<int32_t> rids = to_host_i32(ctx, H.recv_ids.p, H.n_recv);
  for (size_t q = 0; q < H.nbr.size(); ++q)
    for (int64_t k = H.recv_off[q]; k < H.recv_off[q + 1]; ++k) {
      const int64_t j = rids[k] - L.n;
      AFEM_REQUIRE(j >= 0 && j < ng, AFEM_ERR_STATE, "amg: a halo receive id outside the ghost columns");
      gown[j] = H.nbr[q];
      gagg[j] = (int32_t)h[j];
    }
}

// the distributed coarse level of L: this rank's aggregates are its rows, the
// aggregates of its ghosts its ghost columns (numbered neighbour by neighbour,
// each neighbour's in increasing aggregate id), and the coarse halo follows
// from L's: the aggregates of the rows L sends to rank s are what s receives
// from this rank, in the same (increasing id) order on both sides
void build_dist_coarse(Ctx& ctx, Amg& a, AmgLevel& L, int64_t nc, AmgLevel& C)
{
  std::vector<int32_t> gagg, gown;
  ghost_aggregates(ctx, L, gagg, gown);
  const Halo& H = *L.H;
  const std::vector<int32_t> agg = to_host_i32(ctx, L.agg.p, L.n);
  const std::vector<int32_t> sids = to_host_i32(ctx, H.send_ids.p, H.n_send);
  const int nn = (int)H.nbr.size();
  std::vector<int64_t> sc(nn), rc(nn);
  std::vector<int32_t> si, ri;
  std::vector<int32_t> cmap(L.ncol, -1);
  for (int64_t i = 0; i < L.n; ++i) cmap[i] = agg[i];
  int64_t next = nc;
  for (int q = 0; q < nn; ++q) {
    std::vector<int32_t> s;
    for (int64_t k = H.send_off[q]; k < H.send_off[q + 1]; ++k)
      if (agg[sids[k]] >= 0) s.push_back(agg[sids[k]]);
    std::sort(s.begin(), s.end());
    s.erase(std::unique(s.begin(), s.end()), s.end());
    sc[q] = (int64_t)s.size();
    si.insert(si.end(), s.begin(), s.end());
    std::vector<int32_t> r;
    for (int64_t j = 0; j < L.ncol - L.n; ++j)
      if (gown[j] == H.nbr[q] && gagg[j] >= 0) r.push_back(gagg[j]);
    std::sort(r.begin(), r.end());
    r.erase(std::unique(r.begin(), r.end()), r.end());
    rc[q] = (int64_t)r.size();
    for (size_t t = 0; t < r.size(); ++t) ri.push_back((int32_t)(next + (int64_t)t));
    for (int64_t j = 0; j < L.ncol - L.n; ++j)
      if (gown[j] == H.nbr[q] && gagg[j] >= 0)
        cmap[L.n + j] = (int32_t)(next + (std::lower_bound(r.begin(), r.end(), gagg[j]) - r.begin()));
    next += (int64_t)r.size();
  }
  C.own_halo.reset(new Halo());
  halo_setup(*C.own_halo, ctx, a.comm, nn, reinterpret_cast<const int32_t*>(H.nbr.data()), sc.data(), si.data(),
             rc.data(), ri.data());
  C.H = C.own_halo.get();
  C.dist = true;
  DevBuf<int32_t> dmap;
  dmap.alloc(L.ncol > 0 ? L.ncol : 1);
  if (L.ncol) AFEM_HIP(hipMemcpyAsync(dmap.p, cmap.data(), L.ncol * sizeof(int32_t), hipMemcpyHostToDevice, ctx.stream));
  DevBuf<int64_t> row_of;
  DevBuf<int32_t> col;
  DevBuf<double> val;
  const int64_t cnnz = galerkin_coo(ctx, L, dmap.p, L.ncol, 0, nc, next, row_of, col, val);
  coo_to_level(ctx, nc, cnnz, row_of, col, val, C);
  C.ncol = next;
}

// the coarse level of L gathered on every rank: this rank's rows of P^T A P in
// the global coarse numbering (aggregates numbered rank by rank), summed into
// one COO over the ranks (all-reduce of zero-padded arrays: every coarse row is
// one rank's), the same replicated CSR on every rank
void build_gathered(Ctx& ctx, Amg& a, AmgLevel& L, int64_t nc, const std::vector<int64_t>& off, AmgLevel& C)
{
  const int nr = comm_nranks(a.comm), me = comm_rank(a.comm);
  std::vector<int32_t> gagg, gown;
  ghost_aggregates(ctx, L, gagg, gown);
  const std::vector<int32_t> agg = to_host_i32(ctx, L.agg.p, L.n);
  const int64_t NG = off[nr];
  AFEM_REQUIRE(NG < (int64_t(1) << 31), AFEM_ERR_LIMIT, "amg: gathered level above 2^31 rows");
  std::vector<int32_t> cmap(L.ncol, -1);
  for (int64_t i = 0; i < L.n; ++i) cmap[i] = agg[i] >= 0 ? (int32_t)(off[me] + agg[i]) : -1;
  for (int64_t j = 0; j < L.ncol - L.n; ++j)
    if (gown[j] >= 0 && gagg[j] >= 0) cmap[L.n + j] = (int32_t)(off[gown[j]] + gagg[j]);
  DevBuf<int32_t> dmap;
  dmap.alloc(L.ncol > 0 ? L.ncol : 1);
  if (L.ncol) AFEM_HIP(hipMemcpyAsync(dmap.p, cmap.data(), L.ncol * sizeof(int32_t), hipMemcpyHostToDevice, ctx.stream));
  DevBuf<int64_t> row_of;
  DevBuf<int32_t> col;
  DevBuf<double> val;
  const int64_t cnnz = galerkin_coo(ctx, L, dmap.p, L.ncol, 0, nc, NG, row_of, col, val);
  // (galerkin_coo keys agg i + row_base: with row_base 0 the rows are my local
  // aggregate ids; shifted to global ids below)
  std::vector<double> cnt(nr, 0.0);
  cnt[me] = (double)cnnz;
  cnt = allsum_vec(ctx, a, cnt);
  std::vector<int64_t> eoff(nr + 1, 0);
  for (int r = 0; r < nr; ++r) eoff[r + 1] = eoff[r] + (int64_t)cnt[r];
  const int64_t E = eoff[nr];
  std::vector<int64_t> hr(cnnz);
  std::vector<int32_t> hc(cnnz);
  std::vector<double> hv(cnnz);
  if (cnnz) {
    AFEM_HIP(hipMemcpyAsync(hr.data(), row_of.p, cnnz * 8, hipMemcpyDeviceToHost, ctx.stream));
    AFEM_HIP(hipMemcpyAsync(hc.data(), col.p, cnnz * 4, hipMemcpyDeviceToHost, ctx.stream));
    AFEM_HIP(hipMemcpyAsync(hv.data(), val.p, cnnz * 8, hipMemcpyDeviceToHost, ctx.stream));
  }
  ctx.sync();
  std::vector<double> R(E, 0.0), Cc(E, 0.0), V(E, 0.0);
  for (int64_t k = 0; k < cnnz; ++k) {
    R[eoff[me] + k] = (double)(off[me] + hr[k]);
    Cc[eoff[me] + k] = (double)hc[k];
    V[eoff[me] + k] = hv[k];
  }
  R = allsum_vec(ctx, a, std::move(R));
  Cc = allsum_vec(ctx, a, std::move(Cc));
  V = allsum_vec(ctx, a, std::move(V));
  DevBuf<double> dr, dc;
  dr.alloc(E > 0 ? E : 1);
  dc.alloc(E > 0 ? E : 1);
  row_of.alloc(E > 0 ? E : 1);
  col.alloc(E > 0 ? E : 1);
  val.alloc(E > 0 ? E : 1);
  if (E) {
    AFEM_HIP(hipMemcpyAsync(dr.p, R.data(), E * 8, hipMemcpyHostToDevice, ctx.stream));
    AFEM_HIP(hipMemcpyAsync(dc.p, Cc.data(), E * 8, hipMemcpyHostToDevice, ctx.stream));
    AFEM_HIP(hipMemcpyAsync(val.p, V.data(), E * 8, hipMemcpyHostToDevice, ctx.stream));
    hipLaunchKernelGGL(k_amg_coo_unpack, dim3(grid_for(E, 256)), dim3(256), 0, ctx.stream, E, dr.p, dc.p, row_of.p,
                       col.p);
    AFEM_LAUNCHED();
  }
  coo_to_level(ctx, NG, E, row_of, col, val, C);
  C.ncol = NG;
  C.dist = false;
  L.gather_off = off[me];
  L.nc_local = nc;
}

// the identity aggregation of a distributed level (every row its own
// aggregate) and the level gathered whole onto C (build_gathered)
void build_passthrough(Ctx& ctx, Amg& a, AmgLevel& L, AmgLevel& C)
{
  const int64_t n = L.n;
  L.agg.alloc(n > 0 ? n : 1);
  L.mem.alloc(n > 0 ? n : 1);
  L.ap.alloc(n + 1);
  std::vector<int32_t> id(n);
  std::vector<int64_t> ap(n + 1);
  for (int64_t i = 0; i < n; ++i) id[i] = (int32_t)i;
  for (int64_t i = 0; i <= n; ++i) ap[i] = i;
  if (n) {
    AFEM_HIP(hipMemcpyAsync(L.agg.p, id.data(), n * 4, hipMemcpyHostToDevice, ctx.stream));
    AFEM_HIP(hipMemcpyAsync(L.mem.p, id.data(), n * 4, hipMemcpyHostToDevice, ctx.stream));
  }
  AFEM_HIP(hipMemcpyAsync(L.ap.p, ap.data(), (n + 1) * 8, hipMemcpyHostToDevice, ctx.stream));
  ctx.sync();
  const int nr = comm_nranks(a.comm);
  std::vector<double> cnt(nr, 0.0);
  cnt[comm_rank(a.comm)] = (double)n;
  cnt = allsum_vec(ctx, a, cnt);
  std::vector<int64_t> off(nr + 1, 0);
  for (int r = 0; r < nr; ++r) off[r + 1] = off[r] + (int64_t)cnt[r];
  build_gathered(ctx, a, L, n, off, C);
  L.pass = true;
}

bool dense_inverse(Ctx& ctx, Amg& a, AmgLevel& L)
{
  const int m = (int)L.n;
  std::vector<int64_t> rp(m + 1);
  AFEM_HIP(hipMemcpyAsync(rp.data(), L.rp, (m + 1) * 8, hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  std::vector<int32_t> ci(rp[m]);
  std::vector<double> v(rp[m]);
  AFEM_HIP(hipMemcpyAsync(ci.data(), L.ci, rp[m] * 4, hipMemcpyDeviceToHost, ctx.stream));
  AFEM_HIP(hipMemcpyAsync(v.data(), L.v, rp[m] * 8, hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  std::vector<double> A((size_t)m * m, 0.0);
  for (int r = 0; r < m; ++r)
    for (int64_t k = rp[r]; k < rp[r + 1]; ++k) A[(size_t)r * m + ci[k]] += v[k];
  std::vector<double> sc(m);
  for (int i = 0; i < m; ++i) {
    if (!(A[(size_t)i * m + i] > 0)) return false;
    sc[i] = 1.0 / std::sqrt(A[(size_t)i * m + i]);
  }
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < m; ++j) A[(size_t)i * m + j] *= sc[i] * sc[j];
  for (int j = 0; j < m; ++j) {
    double d = A[(size_t)j * m + j];
    for (int q = 0; q < j; ++q) d -= A[(size_t)j * m + q] * A[(size_t)j * m + q];
    if (!(d > 1e-13)) return false;  // singular (no constraint reaches this level's operator): Jacobi sweeps
    d = std::sqrt(d);
    A[(size_t)j * m + j] = d;
    for (int i = j + 1; i < m; ++i) {
      double s = A[(size_t)i * m + j];
      for (int q = 0; q < j; ++q) s -= A[(size_t)i * m + q] * A[(size_t)j * m + q];
      A[(size_t)i * m + j] = s / d;
    }
  }
  std::vector<double> inv((size_t)m * m), y(m);
  for (int c = 0; c < m; ++c) {
    for (int i = 0; i < m; ++i) {
      double s = i == c ? 1.0 : 0.0;
      for (int q = 0; q < i; ++q) s -= A[(size_t)i * m + q] * y[q];
      y[i] = s / A[(size_t)i * m + i];
    }
    for (int i = m - 1; i >= 0; --i) {
      double s = y[i];
      for (int q = i + 1; q < m; ++q) s -= A[(size_t)q * m + i] * y[q];
      y[i] = s / A[(size_t)i * m + i];
    }
    for (int i = 0; i < m; ++i) inv[(size_t)i * m + c] = y[i] * sc[i] * sc[c];
  }
  a.ainv.alloc((size_t)m * m);
  AFEM_HIP(hipMemcpyAsync(a.ainv.p, inv.data(), inv.size() * 8, hipMemcpyHostToDevice, ctx.stream));
  ctx.sync();
  a.n_dense = m;
  return true;
}

// fine: the system whose plan runs the level's products (level 0), else null;
// a distributed level exchanges its iterate's ghosts before every product
void smooth(Ctx& ctx, Amg& a, AmgLevel& L, const double* b, int sweeps, bool from_zero, LinearSystem* fine)
{
  const unsigned g = (unsigned)std::min<int64_t>(kVec, std::max<int64_t>(1, (L.n + 255) / 256));
  int s = 0;
  if (from_zero) {
    if (L.n > 0) {
      hipLaunchKernelGGL(k_amg_scale, dim3(g), dim3(256), 0, ctx.stream, L.n, L.omega, L.dinv.p, b, L.x.p);
      AFEM_LAUNCHED();
    }
    s = 1;
  }
  for (; s < sweeps; ++s) {
    halo(ctx, L, L.x.p);
    if (fine && a.v32.p) {
      f32_product(ctx, a, L, 1, L.x.p, b, L.t.p);
      std::swap(L.x, L.t);
    }
    else if (fine) {
      ls_spmv_planned(*fine, L.x.p, L.t.p);
      hipLaunchKernelGGL(k_amg_jacobi, dim3(g), dim3(256), 0, ctx.stream, L.n, L.omega, L.dinv.p, b, L.t.p, L.x.p);
      AFEM_LAUNCHED();
    }
    else {
      spmv(ctx, 1, L, L.x.p, L.t.p, b, L.omega);
      std::swap(L.x, L.t);
    }
  }
}

void kcycle(Ctx& ctx, Amg& a, size_t l);

// amg_apply's fused entry / exit on level 0 (one rank, fp32 fine copy): the first
// sweep already done by k_amg_mask_scale; the last sweep writes z with the
// constraint rows (k_amg_f32<3>) -- done reports it
struct AmgExit {
  double* z = nullptr;
  const double* r = nullptr;
  const uint8_t* cons = nullptr;
  const double* dfix = nullptr;
  bool done = false;
};

void vcycle(Ctx& ctx, Amg& a, size_t l, const double* b, LinearSystem* fine, AmgExit* ex = nullptr)
{
  AmgLevel& L = a.lv[l];
  if (l > 0) {
    fine = nullptr;
    ex = nullptr;
  }
  if (l + 1 == a.lv.size()) {
    if (a.n_dense == L.n && L.n > 0 && !L.dist) {
      hipLaunchKernelGGL(k_amg_gemv, dim3((unsigned)L.n), dim3(64), 0, ctx.stream, (int)L.n, a.ainv.p, b, L.x.p);
      AFEM_LAUNCHED();
    }
    else {
      smooth(ctx, a, L, b, l == 0 ? 2 * a.sweeps : kCoarseSweeps, true, fine);
    }
    return;
  }
  AmgLevel& C = a.lv[l + 1];
  if (L.pass) {  // gathered whole: C's solution, this rank's part
    AFEM_HIP(hipMemsetAsync(C.b.p, 0, C.n * sizeof(double), ctx.stream));
    if (L.n > 0)
      AFEM_HIP(hipMemcpyAsync(C.b.p + L.gather_off, b, L.n * sizeof(double), hipMemcpyDeviceToDevice, ctx.stream));
    comm_allreduce(a.comm, ctx, C.b.p, C.n);
    if (C.kcoef.p)
      kcycle(ctx, a, l + 1);
    else
      vcycle(ctx, a, l + 1, C.b.p, nullptr);
    if (L.n > 0)
      AFEM_HIP(hipMemcpyAsync(L.x.p, C.x.p + L.gather_off, L.n * sizeof(double), hipMemcpyDeviceToDevice, ctx.stream));
    return;
  }
  if (ex)
    smooth(ctx, a, L, b, a.sweeps - 1, false, fine);  // (the first sweep from zero came with the mask)
  else
    smooth(ctx, a, L, b, a.sweeps, true, fine);
  halo(ctx, L, L.x.p);
  if (fine && a.v32.p) {
    f32_product(ctx, a, L, 2, L.x.p, b, L.r.p);
  }
  else if (fine) {
    ls_spmv_planned(*fine, L.x.p, L.t.p);
    const unsigned gv = (unsigned)std::min<int64_t>(kVec, (L.n + 255) / 256);
    hipLaunchKernelGGL(k_amg_resid, dim3(gv), dim3(256), 0, ctx.stream, L.n, b, L.t.p, L.r.p);
    AFEM_LAUNCHED();
  }
  else {
    spmv(ctx, 2, L, L.x.p, L.r.p, b, 0.0);
  }
  // restriction: into the coarse level's own rows, or (gathered) into this
  // rank's rows of the replicated coarse vector, summed over the ranks
  const bool gathered = L.gather_off >= 0;
  const int64_t nloc = gathered ? L.nc_local : C.n;
  double* cb = C.b.p + (gathered ? L.gather_off : 0);
  if (gathered) AFEM_HIP(hipMemsetAsync(C.b.p, 0, C.n * sizeof(double), ctx.stream));
  if (nloc > 0) {
    hipLaunchKernelGGL(k_amg_restrict, dim3(grid_for(nloc, 256)), dim3(256), 0, ctx.stream, nloc, L.ap.p, L.mem.p,
                       L.r.p, cb);
    AFEM_LAUNCHED();
  }
  if (gathered) comm_allreduce(a.comm, ctx, C.b.p, C.n);
  const bool kc = C.kcoef.p != nullptr;
  if (kc)
    kcycle(ctx, a, l + 1);
  else
    vcycle(ctx, a, l + 1, C.b.p, nullptr);
  if (L.n > 0) {
    const unsigned g = (unsigned)std::min<int64_t>(kVec, (L.n + 255) / 256);
    // (the K-cycle's Krylov weights are the coarse correction's scale)
    hipLaunchKernelGGL(k_amg_prolong, dim3(g), dim3(256), 0, ctx.stream, L.n, L.agg.p, kc ? 1.0 : a.scale,
                       (const double*)(C.x.p + (gathered ? L.gather_off : 0)), L.x.p);
    AFEM_LAUNCHED();
  }
  if (ex) {
    smooth(ctx, a, L, b, a.sweeps - 1, false, fine);
    f32_product(ctx, a, L, 3, L.x.p, b, ex->z, ex->cons, ex->r, ex->dfix);
    ex->done = true;
  }
  else {
    smooth(ctx, a, L, b, a.sweeps, false, fine);
  }
}

// level l's coarse problem A x = b (b in L.b): c1 = B b, v1 = A c1, rt = b -
// alpha1 v1, c2 = B rt, v2 = A c2, x = w1 c1 + w2 c2 (B: the cycle at this
// level); one rank: every scalar stays on the device (graph-capturable, no host
// sync); a distributed level all-reduces the step's dot products
void kcycle(Ctx& ctx, Amg& a, size_t l)
{
  AmgLevel& L = a.lv[l];
  const int64_t n = L.n;
  const unsigned g = (unsigned)std::min<int64_t>(kVec, std::max<int64_t>(1, (n + 255) / 256));
  const unsigned gd = (unsigned)std::min<int64_t>(kDotGrid, std::max<int64_t>(1, (n + 255) / 256));
  auto coef = [&](auto step) {
    constexpr int STEP = decltype(step)::value;
    constexpr int ND = STEP == 1 ? 2 : 3;
    if (!L.dist) {
      hipLaunchKernelGGL(k_kc_coef<STEP>, dim3(1), dim3(256), 0, ctx.stream, (int)gd, (const double*)a.partial.p,
                         L.kcoef.p);
    }
    else {
      hipLaunchKernelGGL(k_kc_sum<ND>, dim3(1), dim3(256), 0, ctx.stream, (int)gd, (const double*)a.partial.p,
                         a.sums.p);
      comm_allreduce(a.comm, ctx, a.sums.p, ND);
      hipLaunchKernelGGL(k_kc_coef_sums<STEP>, dim3(1), dim3(64), 0, ctx.stream, (const double*)a.sums.p, L.kcoef.p);
    }
    AFEM_LAUNCHED();
  };
  vcycle(ctx, a, l, L.b.p, nullptr);
  AFEM_HIP(hipMemcpyAsync(L.kc1.p, L.x.p, n * sizeof(double), hipMemcpyDeviceToDevice, ctx.stream));
  halo(ctx, L, L.kc1.p);
  spmv(ctx, 0, L, L.kc1.p, L.kv1.p, nullptr, 0.0);
  hipLaunchKernelGGL(k_kc_dots<2>, dim3(gd), dim3(256), 0, ctx.stream, n, (const double*)L.kc1.p,
                     (const double*)L.kv1.p, (const double*)L.kc1.p, (const double*)L.b.p, (const double*)nullptr,
                     (const double*)nullptr, a.partial.p);
  AFEM_LAUNCHED();
  coef(std::integral_constant<int, 1>());
  hipLaunchKernelGGL(k_kc_resid, dim3(g), dim3(256), 0, ctx.stream, n, (const double*)L.kcoef.p, (const double*)L.b.p,
                     (const double*)L.kv1.p, L.krt.p);
  AFEM_LAUNCHED();
  vcycle(ctx, a, l, L.krt.p, nullptr);
  halo(ctx, L, L.x.p);
  spmv(ctx, 0, L, L.x.p, L.t.p, nullptr, 0.0);
  hipLaunchKernelGGL(k_kc_dots<3>, dim3(gd), dim3(256), 0, ctx.stream, n, (const double*)L.x.p, (const double*)L.kv1.p,
                     (const double*)L.x.p, (const double*)L.t.p, (const double*)L.x.p, (const double*)L.krt.p,
                     a.partial.p);
  AFEM_LAUNCHED();
  coef(std::integral_constant<int, 2>());
  hipLaunchKernelGGL(k_kc_comb, dim3(g), dim3(256), 0, ctx.stream, n, (const double*)L.kcoef.p,
                     (const double*)L.kc1.p, L.x.p);
  AFEM_LAUNCHED();
}

}  // namespace

bool amg_setup(LinearSystem& ls)
{
  Ctx& ctx = *ls.ctx;
  AFEM_REQUIRE(amg_available(ls), AFEM_ERR_STATE, "amg: needs a CSR system (below 2^31 rows and non-zeros)");
  // amg-reuse: the same CSR arrays at the same sizes (every entry point that
  // installs or rebuilds a matrix also drops ls.amg, capi.cpp / elastodynamics.cpp)
  if (ls.opts.amg == 2 && ls.amg && ls.amg->key_rows == ls.csr_rows && ls.amg->key_cols == ls.csr_cols &&
      ls.amg->key_vals == ls.csr_vals && ls.amg->key_n == ls.n_rows && ls.amg->key_nnz == ls.csr_nnz) {
    f32_refresh(ctx, *ls.amg, ls.amg->lv[0]);  // the fine products follow the live values, as the fp64 ones do
    return false;
  }
  auto a = std::unique_ptr<Amg, AmgDeleter>(new Amg());
  a->partial.alloc(kVec);
  a->sums.alloc(8);
  const bool dist = multi_rank(ls);
  a->comm = dist ? ls.halo->comm : nullptr;
  a->sweeps = (int)std::max(1.0, env_double("AFEM_AMG_SWEEPS", 1.0));
  a->scale = env_double("AFEM_AMG_SCALE", 1.7);
  a->omega_scale = std::min(2.0, std::max(0.1, env_double("AFEM_AMG_OMEGA", 1.0)));
  a->power_its = (int)std::min(200.0, std::max(1.0, env_double("AFEM_AMG_POWER_ITS", kPowerIts)));
  a->fine_planned = env_double("AFEM_AMG_FINE_CSR", 0.0) == 0.0;
  a->use_graph = !dist && env_double("AFEM_AMG_GRAPH", 0.0) != 0.0;
  const double theta = env_double("AFEM_AMG_THETA", 0.05);
  // aggregation distance: level 0 / the coarse levels (distance 1 stalls on the
  // coarse Galerkin graphs: their degree falls with the level, r05w; distance 2
  // everywhere: 108 iterations, 0.44 s with setup, at the unstructured leg's
  // 11.5 M rows against 142 and 0.77 s for 1 / 2, r05aa)
  const int hops0 = (int)std::min(2.0, std::max(1.0, env_double("AFEM_AMG_HOPS0", 2.0)));
  const int hops = (int)std::min(2.0, std::max(1.0, env_double("AFEM_AMG_HOPS", 2.0)));
  const int64_t dense = (int64_t)std::min(4096.0, std::max(1.0, env_double("AFEM_AMG_DENSE", kDense)));
  // several ranks: distributed levels while the global coarse size exceeds
  // AFEM_AMG_GATHER rows, then one level gathered on every rank (its hierarchy
  // below is the one-rank one, built identically on every rank)
  // (at least the dense size: a distributed level never ends the hierarchy
  // below it unless coarsening stalls)
  const int64_t gather_rows = std::max<int64_t>(dense, (int64_t)std::max(1.0, env_double("AFEM_AMG_GATHER", 65536.0)));
  {
    AmgLevel L;
    L.n = ls.n_rows;
    L.ncol = dist ? ls.n_cols : ls.n_rows;
    L.nnz = ls.csr_nnz;
    L.rp = ls.csr_rows;
    L.ci = ls.csr_cols;
    L.v = ls.csr_vals;
    L.dist = dist;
    L.H = dist ? ls.halo.get() : nullptr;
    level_prepare(ctx, L, ls.cons.p);
    a->lv.push_back(std::move(L));
  }
  // AFEM_AMG_F32 (>= 1, default 2; one rank, 16-B aligned CSR arrays, 256-row segments within 64 KB of LDS)
  if (!dist && env_double("AFEM_AMG_F32", 2.0) >= 1.0 && ls.csr_nnz >= 4 && ((uintptr_t)ls.csr_cols & 15) == 0 &&
      ((uintptr_t)ls.csr_vals & 15) == 0) {
    DevBuf<unsigned long long> mx;
    mx.alloc(1);
    AFEM_HIP(hipMemsetAsync(mx.p, 0, mx.bytes(), ctx.stream));
    const int64_t nb = (ls.n_rows + 255) / 256;
    hipLaunchKernelGGL(k_amg_seg256, dim3(grid_for(nb, 256)), dim3(256), 0, ctx.stream, ls.n_rows, ls.csr_rows, mx.p);
    AFEM_LAUNCHED();
    unsigned long long hm = 0;
    AFEM_HIP(hipMemcpyAsync(&hm, mx.p, sizeof(hm), hipMemcpyDeviceToHost, ctx.stream));
    ctx.sync();
    if (hm * 8 + 32 <= 64 * 1024) {
      a->f32_seg = (int64_t)hm;
      a->v32.alloc(ls.csr_nnz);
      f32_refresh(ctx, *a, a->lv[0]);
    }
  }
  const bool verbose = env_double("AFEM_AMG_VERBOSE", 0.0) > 0;
  // AFEM_AMG_VERBOSE: wall time of the setup phases (the device drained at each mark)
  auto t_last = std::chrono::steady_clock::now();
  auto mark = [&](const char* what) {
    if (!verbose) return;
    ctx.sync();
    const auto t = std::chrono::steady_clock::now();
    std::fprintf(stderr, "amg setup %-28s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(t - t_last).count());
    t_last = t;
  };
  mark("fine level");
  while ((int)a->lv.size() < kMaxLevels) {
    AmgLevel& L = a->lv.back();
    const int64_t n_glob = L.dist ? (int64_t)allsum(ctx, *a, (double)L.n) : L.n;
    auto pass = [&]() {  // a small distributed level: gathered whole, solved below
      AmgLevel C;
      build_passthrough(ctx, *a, L, C);
      level_prepare(ctx, C, nullptr);
      a->lv.push_back(std::move(C));
    };
    if (n_glob <= dense) {
      if (!L.dist) break;
      pass();
      continue;
    }
    const int64_t nc = aggregate(ctx, L, theta, a->lv.size() == 1 ? hops0 : hops);
    mark("aggregate");
    const int64_t nc_glob = L.dist ? (int64_t)allsum(ctx, *a, (double)nc) : nc;
    if (verbose)
      std::fprintf(stderr, "amg level %zu%s: %lld rows, %lld non-zeros -> %lld aggregates (global %lld -> %lld)\n",
                   a->lv.size() - 1, L.dist ? " (distributed)" : "", (long long)L.n, (long long)L.nnz, (long long)nc,
                   (long long)n_glob, (long long)nc_glob);
    if (nc_glob == 0 || nc_glob * 10 > n_glob * 9) {  // no coarse level, or coarsening stalls (every rank agrees)
      L.agg.reset();
      L.ap.reset();
      L.mem.reset();
      if (L.dist && n_glob <= gather_rows) {  // gathered whole: its one-rank hierarchy below
        pass();
        continue;
      }
      break;
    }
    AmgLevel C;
    if (!L.dist) {
      galerkin(ctx, L, nc, C);
    }
    else if (nc_glob <= gather_rows) {
      const int nr = comm_nranks(a->comm);
      std::vector<double> cnt(nr, 0.0);
      cnt[comm_rank(a->comm)] = (double)nc;
      cnt = allsum_vec(ctx, *a, cnt);
      std::vector<int64_t> off(nr + 1, 0);
      for (int r = 0; r < nr; ++r) off[r + 1] = off[r] + (int64_t)cnt[r];
      build_gathered(ctx, *a, L, nc, off, C);
    }
    else {
      build_dist_coarse(ctx, *a, L, nc, C);
    }
    mark("coarse operator");
    level_prepare(ctx, C, nullptr);
    a->lv.push_back(std::move(C));
    mark("coarse level prepared");
  }
  for (auto& L : a->lv) {
    // the power iteration approaches lambda_max from below: 10 % margin (an
    // underestimate by 1.5x would make the smoother diverge)
    const double lam = 1.1 * power_lambda(ctx, *a, L);
    L.omega = lam > 0 ? a->omega_scale * 4.0 / (3.0 * lam) : 0.0;
  }
  mark("power iterations");
  AmgLevel& last = a->lv.back();
  // the coarsest level inverted densely when small (a small system: the
  // whole matrix, the PCG then converges in one or two iterations); a
  // distributed coarsest level (no gathered one below) is smoothed
  if (!last.dist && last.n <= dense) dense_inverse(ctx, *a, last);
  // K-cycle on levels 1 and 2 (the unstructured leg's 11.5 M rows, r05ay: 108 -> 72
  // iterations, 0.453 -> 0.389 s with setup; every level: 66, 0.407 s -- the small
  // levels' launches, visited 2^l times, cost more than the iterations they save)
  a->kcycle = (int)std::max(0.0, env_double("AFEM_AMG_KCYCLE", 2.0));
  for (size_t l = 1; l < a->lv.size() && (int)l <= a->kcycle; ++l) {
    AmgLevel& L = a->lv[l];
    if (l + 1 == a->lv.size() && a->n_dense == L.n && !L.dist) break;  // the dense coarsest level: solved exactly
    L.kc1.alloc(L.ncol > 0 ? L.ncol : 1);
    AFEM_HIP(hipMemsetAsync(L.kc1.p, 0, L.kc1.bytes(), ctx.stream));
    L.kv1.alloc(L.n > 0 ? L.n : 1);
    L.krt.alloc(L.n > 0 ? L.n : 1);
    L.kcoef.alloc(8);
  }
  // AFEM_AMG_F32 = 2 (the default): the coarse levels' cycle and K-cycle products on fp32
  // copies of their values (fixed with the hierarchy; the power iterations above ran on fp64)
  if (env_double("AFEM_AMG_F32", 2.0) >= 2.0) {
    for (size_t l = 1; l < a->lv.size(); ++l) {
      AmgLevel& L = a->lv[l];
      if (L.nnz <= 0 || !L.v) continue;
      L.v32.alloc(L.nnz);
      hipLaunchKernelGGL(k_amg_d2f, dim3((unsigned)std::min<int64_t>(kVec, (L.nnz + 255) / 256)), dim3(256), 0,
                         ctx.stream, L.nnz, L.v, L.v32.p);
      AFEM_LAUNCHED();
    }
  }
  mark("dense coarsest, K-cycle buffers");
  a->key_rows = ls.csr_rows;
  a->key_cols = ls.csr_cols;
  a->key_vals = ls.csr_vals;
  a->key_n = ls.n_rows;
  a->key_nnz = ls.csr_nnz;
  ls.amg = std::move(a);
  return true;
}

namespace {
void amg_apply_launch(LinearSystem& ls, const double* r, double* z);
}

void amg_apply(LinearSystem& ls, const double* r, double* z)
{
  Ctx& ctx = *ls.ctx;
  Amg& a = *ls.amg;
  if (!a.use_graph) {
    amg_apply_launch(ls, r, z);
    return;
  }
  if (!a.gexec || a.g_r != r || a.g_z != z || a.g_plan != ls.spmv_plan.get()) {
    if (a.gexec) {
      AFEM_HIP(hipGraphExecDestroy(a.gexec));
      a.gexec = nullptr;
    }
    hipGraph_t graph = nullptr;
    AFEM_HIP(hipStreamBeginCapture(ctx.stream, hipStreamCaptureModeThreadLocal));
    try {
      amg_apply_launch(ls, r, z);
    }
    catch (...) {
      (void)hipStreamEndCapture(ctx.stream, &graph);
      if (graph) (void)hipGraphDestroy(graph);
      throw;
    }
    AFEM_HIP(hipStreamEndCapture(ctx.stream, &graph));
    const hipError_t e = hipGraphInstantiate(&a.gexec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    AFEM_HIP(e);
    a.g_r = r;
    a.g_z = z;
    a.g_plan = ls.spmv_plan.get();
  }
  AFEM_HIP(hipGraphLaunch(a.gexec, ctx.stream));
}

namespace {
void amg_apply_launch(LinearSystem& ls, const double* r, double* z)
{
  Ctx& ctx = *ls.ctx;
  Amg& a = *ls.amg;
  AmgLevel& L0 = a.lv[0];
  const int64_t n = ls.n_rows;
  const unsigned g = (unsigned)std::min<int64_t>(kVec, (n + 255) / 256);
  LinearSystem* fine = a.fine_planned && ls.spmv_plan ? &ls : nullptr;
  // one rank with the fp32 fine copy and a coarse level: the entry (mask + first sweep) and the exit
  // (last sweep into z + constraint rows) fused (AFEM_AMG_FUSE=0: separate passes)
  if (fine && a.v32.p && a.lv.size() > 1 && !L0.dist && L0.n == n && a.sweeps >= 1 &&
      env_double("AFEM_AMG_FUSE", 1.0) != 0.0) {
    hipLaunchKernelGGL(k_amg_mask_scale, dim3(g), dim3(256), 0, ctx.stream, n, ls.cons.p, r, L0.omega,
                       (const double*)L0.dinv.p, L0.b.p, L0.x.p);
    AFEM_LAUNCHED();
    AmgExit ex;
    ex.z = z;
    ex.r = r;
    ex.cons = ls.cons.p;
    ex.dfix = ls.dinv.p;
    vcycle(ctx, a, 0, L0.b.p, fine, &ex);
    if (ex.done) return;
  }
  else {
    hipLaunchKernelGGL(k_amg_mask, dim3(g), dim3(256), 0, ctx.stream, n, ls.cons.p, r, L0.b.p);
    AFEM_LAUNCHED();
    // the fine level's products through the PCG's SpMV plan (AFEM_AMG_FINE_CSR=1: the 8-lane CSR kernel)
    vcycle(ctx, a, 0, L0.b.p, fine);
  }
  AFEM_HIP(hipMemcpyAsync(z, L0.x.p, n * sizeof(double), hipMemcpyDeviceToDevice, ctx.stream));
  hipLaunchKernelGGL(k_amg_fix, dim3(g), dim3(256), 0, ctx.stream, n, ls.cons.p, r, ls.dinv.p, z);
  AFEM_LAUNCHED();
}
}  // namespace

void amg_stats(const LinearSystem& ls, int32_t* levels, int64_t* coarse_rows, double* complexity)
{
  if (!ls.amg) {
    *levels = 0;
    *coarse_rows = 0;
    *complexity = 0.0;
    return;
  }
  *levels = (int32_t)ls.amg->lv.size();
  *coarse_rows = ls.amg->lv.back().n;
  double nz = 0.0;
  for (const auto& L : ls.amg->lv) nz += (double)L.nnz;
  *complexity = ls.amg->lv[0].nnz > 0 ? nz / (double)ls.amg->lv[0].nnz : 0.0;
}

}  // namespace afem
