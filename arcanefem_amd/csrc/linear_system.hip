// DoFLinearSystemImpl on the GPU: boundary-condition kernels (K16-K19 of
// SURVEY.md §2.4), the Jacobi-preconditioned CG whose SpMV reuses the
// assembled CSR (replaces Hypre PCG+BoomerAMG / the Sequential MatVec CG,
// femutils/HypreDoFLinearSystem.cc:387-762, femutils/DoFLinearSystem.cc:106-164),
// and the host COO path for modules that call matrixAddValue entry by entry
// (Aleph semantics, femutils/AlephDoFLinearSystem.cc:192-223,501-583).
#include "afem_internal.hpp"

#include <functional>

#include <chrono>

#include <cstdio>
#include <cstdlib>
#include <string>

#include <cmath>
#include <cstring>
#include <algorithm>
#include <vector>

namespace afem {
namespace {

constexpr int kThreads = 256;
inline unsigned grid_for(int64_t n, int threads) { return (unsigned)((n + threads - 1) / threads); }
constexpr uint8_t kElimRow = 1, kElimRowCol = 2;

// ---------------------------------------------------------------- BC kernels
// kind 0: penalty  (femutils/ArcaneFemFunctionsGpu.h:434-456)
// kind 1: row elimination, kind 2: row+column elimination (:461-482)
// values (may be null): one value per listed DoF instead of the common `value`
__global__ void k_set_list(int64_t n, const int32_t* __restrict__ ids, int kind, double value,
                           const double* __restrict__ values, double penalty, int64_t n_rows,
                           uint8_t* __restrict__ forced_info, double* __restrict__ forced_value,
                           uint8_t* __restrict__ elim_info, double* __restrict__ elim_value, double* __restrict__ rhs)
{
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  int32_t d = ids[t];
  if (d < 0 || d >= n_rows) return;  // isOwn() filter
  if (values) value = values[t];
  if (kind == 0) {
    forced_info[d] = 1;
    forced_value[d] = penalty;
    rhs[d] = penalty * value;
  }
  else {
    elim_info[d] = (kind == 1) ? kElimRow : kElimRowCol;
    elim_value[d] = value;
  }
}

// Row+column elimination, phase 1 (Aleph _fillMatrix,
// femutils/AlephDoFLinearSystem.cc:539-565): for every row+column eliminated
// DoF i and every owned column j != i of row i, rhs_j -= A[i,j] * g_i (the
// eliminated ROW's entry), and the column entries A[j,i] of the other rows
// are dropped.  Gathered per row j (no atomics, fixed summation order): the
// eliminated rows coupled to j are the RC-eliminated columns of row j (the
// P1 structure is symmetric), A[i,j] is looked up in row i.  Eliminated rows
// are skipped (their rhs is overwritten by g in phase 2) and not modified
// here, so the lookups read final values.
__global__ void k_elim_columns(int64_t n_rows, const int64_t* __restrict__ rows, const int32_t* __restrict__ cols,
                               double* __restrict__ vals, const uint8_t* __restrict__ elim_info,
                               const double* __restrict__ elim_value, double* __restrict__ rhs)
{
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_rows) return;
  if (elim_info[j] != 0) return;
  double acc = 0.0;
  for (int64_t k = rows[j]; k < rows[j + 1]; ++k) {
    int32_t i = cols[k];
    if (i != (int32_t)j && i < n_rows && elim_info[i] == kElimRowCol) {
      double a_ij = 0.0;
      for (int64_t t = rows[i]; t < rows[i + 1]; ++t)
        if (cols[t] == (int32_t)j) {
          a_ij = vals[t];
          break;
        }
      acc += a_ij * elim_value[i];
      vals[k] = 0.0;
    }
  }
  if (acc != 0.0) rhs[j] -= acc;
}

// _applyRowElimination then _applyForcedValuesToLhs
// (femutils/HypreDoFLinearSystem.cc:319-382).
// 4 rows per thread: the two flag arrays read as one 32-bit word each (a
// thread per row was bound by wave launches; 16 rows per thread serialised the
// flagged rows of a Dirichlet face: 51 us; a persistent grid-stride sweep: no
// better), the diagonal of a forced row from the BSRFormat's diagonal
// positions when the view is its CSR, else found by a binary search of the
// sorted row (a linear scan for unsorted views)
__global__ void k_apply_bcs(int64_t n_rows, const int64_t* __restrict__ rows, const int32_t* __restrict__ cols,
                            double* __restrict__ vals, const uint8_t* __restrict__ forced_info,
                            const double* __restrict__ forced_value, const uint8_t* __restrict__ elim_info,
                            const double* __restrict__ elim_value, double* __restrict__ rhs,
                            const int64_t* __restrict__ diag)
{
  const int64_t d0 = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (d0 >= n_rows) return;
  uint32_t fw = 0, ew = 0;
  if (d0 + 4 <= n_rows) {
    fw = *reinterpret_cast<const uint32_t*>(forced_info + d0);
    ew = *reinterpret_cast<const uint32_t*>(elim_info + d0);
  }
  else {
    for (int i = 0; d0 + i < n_rows; ++i) {
      fw |= (uint32_t)forced_info[d0 + i] << (8 * i);
      ew |= (uint32_t)elim_info[d0 + i] << (8 * i);
    }
  }
  if (!(fw | ew)) return;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bool ei = (ew >> (8 * i)) & 0xFFu, fi = (fw >> (8 * i)) & 0xFFu;
    if (!ei && !fi) continue;
    const int64_t d = d0 + i;
    if (fi && !ei && diag) {
      vals[diag[d]] = forced_value[d];
      continue;
    }
    const int64_t b = rows[d], e = rows[d + 1];
    if (ei) {
      for (int64_t k = b; k < e; ++k) vals[k] = (cols[k] == (int32_t)d) ? 1.0 : 0.0;
      rhs[d] = elim_value[d];
    }
    if (fi && diag) {  // the view is a BSRFormat's own CSR: its diagonal positions
      vals[diag[d]] = forced_value[d];
    }
    else if (fi) {
      int64_t lo = b, hi = e;  // lower bound of d (sorted rows)
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (cols[mid] < (int32_t)d)
          lo = mid + 1;
        else
          hi = mid;
      }
      if (lo < e && cols[lo] == (int32_t)d)
        vals[lo] = forced_value[d];
      else
        for (int64_t k = b; k < e; ++k)  // an unsorted view
          if (cols[k] == (int32_t)d) {
            vals[k] = forced_value[d];
            break;
          }
    }
  }
}

__global__ void k_point_update(const int64_t* __restrict__ rows, const int32_t* __restrict__ cols,
                               double* __restrict__ vals, int32_t row, int32_t col, double v, int set,
                               int32_t* __restrict__ found)
{
  if (threadIdx.x != 0) return;
  for (int64_t k = rows[row]; k < rows[row + 1]; ++k)
    if (cols[k] == col) {
      if (set)
        vals[k] = v;
      else
        vals[k] += v;
      *found = 1;
      return;
    }
  *found = 0;
}

// ---------------------------------------------------------------- CG kernels
__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += __shfl_down(v, d, 64);
  return v;
}

__device__ __forceinline__ double block_sum(double v)
{
  __shared__ double ws[kThreads / 64];
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) ws[wid] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0) {
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += ws[w];
  }
  __syncthreads();
  return s;  // valid in thread 0
}

__device__ __forceinline__ int64_t xcd_swizzle(int64_t b, int64_t nb)
{
  const int64_t q = nb >> 3, rem = nb & 7;
  const int64_t x = b & 7, i = b >> 3;
  return x * q + (x < rem ? x : rem) + i;
}

// CSR SpMV y = A x over a block of rows (CSR-stream: the block's contiguous
// value/column segment is read with coalesced loads, products staged in LDS,
// one lane per row reduces its products).  DOT: block partial of x[r]*y[r].
template <bool DOT>
__global__ __launch_bounds__(kThreads) void k_spmv_stream(int64_t n_rows, const int64_t* __restrict__ rows,
                                                          const int32_t* __restrict__ cols,
                                                          const double* __restrict__ vals,
                                                          const double* __restrict__ x, double* __restrict__ y,
                                                          double* __restrict__ partial)
{
  extern __shared__ __align__(16) unsigned char smem[];
  double* prod = reinterpret_cast<double*>(smem);
  const int rpb = blockDim.x;
  const int64_t blk = xcd_swizzle(blockIdx.x, gridDim.x);
  const int64_t r0 = blk * rpb;
  const int64_t r1 = (r0 + rpb < n_rows) ? r0 + rpb : n_rows;
  const int64_t seg0 = rows[r0], seglen = rows[r1] - seg0;
  for (int64_t t = threadIdx.x; t < seglen; t += rpb) prod[t] = vals[seg0 + t] * x[cols[seg0 + t]];
  __syncthreads();
  const int64_t r = r0 + threadIdx.x;
  double d = 0.0;
  if (r < r1) {
    double s = 0.0;
    for (int64_t k = rows[r] - seg0, e = rows[r + 1] - seg0; k < e; ++k) s += prod[k];
    y[r] = s;
    if (DOT) d = x[r] * s;
  }
  if (DOT) {
    double bs = block_sum(d);
    if (threadIdx.x == 0) partial[blockIdx.x] = bs;
  }
}

// CSR-stream with 16-B loads: the block's value/column segment is read as
// aligned groups of 4 non-zeros (one dwordx4 of columns and two dwordx4 of
// values per lane: 0.75 vector-memory address ops per non-zero instead of 2),
// the 4 gathers of x are issued together, products go to LDS; then one lane
// per row sums its run (as k_spmv_stream).  Needs 16-B aligned cols/vals
// bases (checked by the planner); the group past nnz is loaded element by
// element.
template <bool DOT>
__global__ __launch_bounds__(kThreads) void k_spmv_stream4(int64_t n_rows, int64_t nnz,
                                                           const int64_t* __restrict__ rows,
                                                           const int32_t* __restrict__ cols,
                                                           const double* __restrict__ vals,
                                                           const double* __restrict__ x, double* __restrict__ y,
                                                           double* __restrict__ partial)
{
  extern __shared__ __align__(16) unsigned char smem[];
  double* prod = reinterpret_cast<double*>(smem);
  const int64_t blk = xcd_swizzle(blockIdx.x, gridDim.x);
  const int64_t r0 = blk * kThreads;
  const int64_t r1 = (r0 + kThreads < n_rows) ? r0 + kThreads : n_rows;
  const int64_t a = rows[r0], b = rows[r1];
  for (int64_t q = (a & ~int64_t(3)) + 4 * (int64_t)threadIdx.x; q < b; q += 4 * kThreads) {
    int c[4];
    double v[4];
    if (q + 4 <= nnz) {
      const int4 c4 = *reinterpret_cast<const int4*>(cols + q);
      const double2 v01 = *reinterpret_cast<const double2*>(vals + q);
      const double2 v23 = *reinterpret_cast<const double2*>(vals + q + 2);
      c[0] = c4.x;
      c[1] = c4.y;
      c[2] = c4.z;
      c[3] = c4.w;
      v[0] = v01.x;
      v[1] = v01.y;
      v[2] = v23.x;
      v[3] = v23.y;
    }
    else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        c[j] = q + j < nnz ? cols[q + j] : 0;
        v[j] = q + j < nnz ? vals[q + j] : 0.0;
      }
    }
    double xv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) xv[j] = x[c[j]];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (q + j >= a && q + j < b) prod[q + j - a] = v[j] * xv[j];
  }
  __syncthreads();
  const int64_t r = r0 + threadIdx.x;
  double d = 0.0;
  if (r < r1) {
    double s = 0.0;
    for (int64_t k = rows[r] - a, e = rows[r + 1] - a; k < e; ++k) s += prod[k];
    y[r] = s;
    if (DOT) d = x[r] * s;
  }
  if (DOT) {
    double bs = block_sum(d);
    if (threadIdx.x == 0) partial[blockIdx.x] = bs;
  }
}

// k_spmv_stream4 with the segment's first kSpmvU groups per lane issued
// together (all column/value loads, then all gathers): kSpmvU round trips of
// memory latency overlap instead of running back to back (a 256-row block of
// 15-non-zero rows is ~4 groups per lane).  Longer segments finish in the
// k_spmv_stream4 loop.
constexpr int kSpmvU = 4;
template <bool DOT, int BS = kThreads>
__global__ __launch_bounds__(BS) void k_spmv_stream4u(int64_t n_rows, int64_t nnz,
                                                            const int64_t* __restrict__ rows,
                                                            const int32_t* __restrict__ cols,
                                                            const double* __restrict__ vals,
                                                            const double* __restrict__ x, double* __restrict__ y,
                                                            double* __restrict__ partial,
                                                            const int32_t* __restrict__ blist = nullptr)
{
  extern __shared__ __align__(16) unsigned char smem[];
  double* prod = reinterpret_cast<double*>(smem);
  // blist: the row blocks of this launch (the CG's interior / halo-boundary split)
  const int64_t blk = blist ? (int64_t)blist[blockIdx.x] : xcd_swizzle(blockIdx.x, gridDim.x);
  const int64_t r0 = blk * BS;
  const int64_t r1 = (r0 + BS < n_rows) ? r0 + BS : n_rows;
  const int64_t a = rows[r0], b = rows[r1];
  const int64_t q0 = (a & ~int64_t(3)) + 4 * (int64_t)threadIdx.x;
  auto load4 = [&](int64_t q, int (&c)[4], double (&v)[4]) {
    if (q + 4 <= nnz) {
      const int4 c4 = *reinterpret_cast<const int4*>(cols + q);
      const double2 v01 = *reinterpret_cast<const double2*>(vals + q);
      const double2 v23 = *reinterpret_cast<const double2*>(vals + q + 2);
      c[0] = c4.x;
      c[1] = c4.y;
      c[2] = c4.z;
      c[3] = c4.w;
      v[0] = v01.x;
      v[1] = v01.y;
      v[2] = v23.x;
      v[3] = v23.y;
    }
    else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        c[j] = q + j < nnz ? cols[q + j] : 0;
        v[j] = q + j < nnz ? vals[q + j] : 0.0;
      }
    }
  };
  // products to LDS: a lane's 4 products are contiguous (32 B), so lanes
  // l, l+8, l+16, l+24 hit the same banks; the t-th store of lane l writes
  // product (t + l/8) mod 4 instead, which spreads them (conflict-free)
  const int rot = (int)(threadIdx.x >> 3) & 3;
  auto put4 = [&](int64_t q, const double (&v)[4], const double (&xv)[4]) {
    double pr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) pr[j] = v[j] * xv[j];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int j = (t + rot) & 3;
      const double w = j == 0 ? pr[0] : (j == 1 ? pr[1] : (j == 2 ? pr[2] : pr[3]));
      if (q + j >= a && q + j < b) prod[q + j - a] = w;
    }
  };
  {
    int c[kSpmvU][4];
    double v[kSpmvU][4];
#pragma unroll
    for (int u = 0; u < kSpmvU; ++u) {
      const int64_t q = q0 + (int64_t)u * 4 * BS;
      if (q < b) {
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
    double xv[kSpmvU][4];
#pragma unroll
    for (int u = 0; u < kSpmvU; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) xv[u][j] = x[c[u][j]];
#pragma unroll
    for (int u = 0; u < kSpmvU; ++u) put4(q0 + (int64_t)u * 4 * BS, v[u], xv[u]);
  }
  for (int64_t q = q0 + (int64_t)kSpmvU * 4 * BS; q < b; q += 4 * BS) {
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
  double d = 0.0;
  if (r < r1) {
    double s = 0.0;
    for (int64_t k = rows[r] - a, e = rows[r + 1] - a; k < e; ++k) s += prod[k];
    y[r] = s;
    if (DOT) d = x[r] * s;
  }
  if (DOT) {
    double bs = block_sum(d);
    if (threadIdx.x == 0) partial[blockIdx.x] = bs;
  }
}

// Vector CSR SpMV: a 16-lane group per row, RPG rows per group with all of
// their loads issued before any use (memory-level parallelism without LDS or
// barriers).  Lane k of a row loads non-zero k (coalesced: a wave's 4 groups
// read ~4*RPG consecutive rows' segments), gathers x, and the row sum is a
// 16-lane shuffle reduction.  Rows longer than 16 loop in 16-wide chunks.
// DOT: block partial of x[r] * y[r] (the CG's p.q).
constexpr int kSpmvRpg = 4;
template <bool DOT>
__global__ __launch_bounds__(256) void k_spmv_v16(int64_t n_rows, const int64_t* __restrict__ rows,
                                                  const int32_t* __restrict__ cols, const double* __restrict__ vals,
                                                  const double* __restrict__ x, double* __restrict__ y,
                                                  double* __restrict__ partial)
{
  const int l16 = threadIdx.x & 15;
  const int64_t g = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
  const int64_t r0 = g * kSpmvRpg;
  int64_t rb[kSpmvRpg], re[kSpmvRpg];
#pragma unroll
  for (int i = 0; i < kSpmvRpg; ++i) {
    const int64_t r = r0 + i < n_rows ? r0 + i : n_rows - 1;
    rb[i] = rows[r];
    re[i] = r0 + i < n_rows ? rows[r + 1] : rb[i];
  }
  double s[kSpmvRpg];
  int32_t c[kSpmvRpg];
  double v[kSpmvRpg];
#pragma unroll
  for (int i = 0; i < kSpmvRpg; ++i) {
    const int64_t k = rb[i] + l16;
    const bool in = k < re[i];
    const int64_t kk = in ? k : rb[i];
    c[i] = cols[kk];
    v[i] = in ? vals[kk] : 0.0;
  }
#pragma unroll
  for (int i = 0; i < kSpmvRpg; ++i) s[i] = v[i] * x[c[i]];
#pragma unroll
  for (int i = 0; i < kSpmvRpg; ++i)
    for (int64_t k = rb[i] + 16 + l16; k < re[i]; k += 16) s[i] += vals[k] * x[cols[k]];
#pragma unroll
  for (int i = 0; i < kSpmvRpg; ++i) {
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) s[i] += __shfl_xor(s[i], o, 16);
  }
  double d = 0.0;
  if (l16 < kSpmvRpg) {
    // lane i of the group writes row r0+i (4 consecutive rows: one 32-B store)
    double si = s[0];
#pragma unroll
    for (int i = 1; i < kSpmvRpg; ++i)
      if (l16 == i) si = s[i];
    const int64_t r = r0 + l16;
    if (r < n_rows) {
      y[r] = si;
      if (DOT) d = x[r] * si;
    }
  }
  if (DOT) {
    double bs = block_sum(d);
    if (threadIdx.x == 0) partial[blockIdx.x] = bs;
  }
}

// Pattern-compressed column indices for the CG's SpMV.  A structured mesh
// numbers its nodes lexicographically, so the interior rows of a Kuhn box have
// the same column offsets c - r (15 of them).  PatOff holds the offsets of
// one interior row; flag[r] = 1 marks every row whose columns are r + off[k],
// k < len (k_pat_flags, once per solve): the SpMV forms those columns instead
// of reading them (4 of the ~13 B per non-zero), the other rows read theirs.
// Values, their order and the summation order are the CSR's: y is bitwise
// the k_spmv_v16 result.
struct PatOff {
  int32_t len;
  int32_t off[16];
};

// 16 lanes per row (coalesced column reads; one thread per row: 18.7 ms at C4):
// lane k compares column k with r + off[k].  A grid-stride loop: one counter
// atomic per wave at the end (an atomic per wave of 4 rows, 25 M at C4, took
// 300 ms on the one address)
__global__ __launch_bounds__(256) void k_pat_flags(int64_t n_rows, const int64_t* __restrict__ rows,
                                                   const int32_t* __restrict__ cols, PatOff po,
                                                   uint8_t* __restrict__ flag, unsigned long long* __restrict__ count)
{
  const int l16 = threadIdx.x & 15;
  int32_t my_off = 0;  // off[l16] (a select chain: no dynamic index into the argument)
#pragma unroll
  for (int k = 0; k < 16; ++k)
    if (k == l16) my_off = po.off[k];
  const int g = (int)(threadIdx.x & 63) & ~15;  // this row group's 16 lanes in the wave
  const int64_t stride = (int64_t)gridDim.x * blockDim.x / 16;
  unsigned long long n_ok = 0;
  for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;; r += stride) {
    // wave-uniform exit (lane 0 holds the wave's first row): the ballots below see all 64 lanes
    if (__shfl(r, 0) >= n_rows) break;
    bool bad = r >= n_rows;
    if (!bad) {
      const int64_t a = rows[r];
      if (rows[r + 1] - a != po.len)
        bad = true;
      else if (l16 < po.len)
        bad = (int64_t)cols[a + l16] != r + my_off;
    }
    const unsigned long long m = __ballot(bad);
    const bool ok = ((m >> g) & 0xFFFFull) == 0;
    if (l16 == 0 && r < n_rows) flag[r] = ok ? 1 : 0;
    n_ok += __popcll(__ballot(l16 == 0 && r < n_rows && ok));
  }
  if ((threadIdx.x & 63) == 0 && n_ok) atomicAdd(count, n_ok);
}

// k_spmv_stream4u with the block's column indices formed in LDS first: the
// thread of a pattern row writes r + off[k] for its row's positions, the
// thread of any other row copies its columns from memory; the stream then
// reads 4 columns per lane from LDS (ds_read_b128) instead of HBM.  Products,
// their order and the row sums are k_spmv_stream4u's (bitwise equal y).
// sample t of 256 rows spread over the range: its length and (<= 16) column offsets
__global__ void k_pat_sample(int64_t n_rows, const int64_t* __restrict__ rows, const int32_t* __restrict__ cols,
                             int32_t* __restrict__ out)
{
  const int t = threadIdx.x;
  const int64_t r = (int64_t)(t + 1) * n_rows / (blockDim.x + 2);
  const int64_t a = rows[r], len = rows[r + 1] - a;
  out[17 * t] = (int32_t)(len <= 16 ? len : 0);
  for (int k = 0; k < 16; ++k) out[17 * t + 1 + k] = k < len ? (int32_t)(cols[a + k] - r) : 0;
}

template <bool DOT, int BS = kThreads>
__global__ __launch_bounds__(BS) void k_spmv_pat(int64_t n_rows, int64_t nnz, const int64_t* __restrict__ rows,
                                                       const int32_t* __restrict__ cols,
                                                       const double* __restrict__ vals,
                                                       const uint8_t* __restrict__ flag, PatOff po,
                                                       const double* __restrict__ x, double* __restrict__ y,
                                                       double* __restrict__ partial, int64_t max_seg,
                                                       const int32_t* __restrict__ blist = nullptr)
{
  extern __shared__ __align__(16) unsigned char smem[];
  double* prod = reinterpret_cast<double*>(smem);
  // the column image [q - (a & ~3)] overlays the products (every column is in
  // registers before the first product is stored: segments <= kSpmvU groups)
  int32_t* cl = reinterpret_cast<int32_t*>(smem);
  // blist: the row blocks of this launch (the CG's interior / halo-boundary split)
  const int64_t blk = blist ? (int64_t)blist[blockIdx.x] : xcd_swizzle(blockIdx.x, gridDim.x);
  const int64_t r0 = blk * BS;
  const int64_t r1 = (r0 + BS < n_rows) ? r0 + BS : n_rows;
  const int64_t a = rows[r0], b = rows[r1];
  const int64_t a4 = a & ~int64_t(3);
  const int64_t r = r0 + threadIdx.x;
  int64_t ra = 0, re = 0;
  if (r < r1) {
    ra = rows[r];
    re = rows[r + 1];
    if (flag[r]) {
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (k < po.len) cl[ra - a4 + k] = (int32_t)r + po.off[k];
    }
    else {
      for (int64_t k = ra; k < re; ++k) cl[k - a4] = cols[k];
    }
  }
  __syncthreads();
  const int64_t q0 = a4 + 4 * (int64_t)threadIdx.x;
  auto load4 = [&](int64_t q, int (&c)[4], double (&v)[4]) {
    const int4 c4 = *reinterpret_cast<const int4*>(cl + (q - a4));
    c[0] = q >= a ? c4.x : 0;
    c[1] = q + 1 >= a && q + 1 < b ? c4.y : 0;
    c[2] = q + 2 >= a && q + 2 < b ? c4.z : 0;
    c[3] = q + 3 >= a && q + 3 < b ? c4.w : 0;
    if (q + 4 <= nnz) {
      const double2 v01 = *reinterpret_cast<const double2*>(vals + q);
      const double2 v23 = *reinterpret_cast<const double2*>(vals + q + 2);
      v[0] = v01.x;
      v[1] = v01.y;
      v[2] = v23.x;
      v[3] = v23.y;
    }
    else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = q + j < nnz ? vals[q + j] : 0.0;
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
      if (q + j >= a && q + j < b) prod[q + j - a] = w;
    }
  };
  {
    int c[kSpmvU][4];
    double v[kSpmvU][4];
#pragma unroll
    for (int u = 0; u < kSpmvU; ++u) {
      const int64_t q = q0 + (int64_t)u * 4 * BS;
      if (q < b) {
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
    double xv[kSpmvU][4];
#pragma unroll
    for (int u = 0; u < kSpmvU; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) xv[u][j] = x[c[u][j]];
    __syncthreads();  // every column read before the products overwrite the column image
#pragma unroll
    for (int u = 0; u < kSpmvU; ++u) put4(q0 + (int64_t)u * 4 * BS, v[u], xv[u]);
  }
  __syncthreads();
  double d = 0.0;
  if (r < r1) {
    double s = 0.0;
    for (int64_t k = ra - a, e = re - a; k < e; ++k) s += prod[k];
    y[r] = s;
    if (DOT) d = x[r] * s;
  }
  if (DOT) {
    double bs = block_sum(d);
    if (threadIdx.x == 0) partial[blockIdx.x] = bs;
  }
}

// Node-block SpMV of an NB_DOF = K system held in BSRFormat's CSR order
// (femutils/BSRFormat.h:194-256: scalar row K r + i holds the node row's
// K * len values as [block s][j]).  The node-row structure (block offsets bp,
// node columns bc) replaces the scalar column indices: 4 B per block instead
// of 4 K^2 B, so a block-3 SpMV reads 76 B per block instead of 108 B.
// 16 lanes per node row (lane t: blocks t, t + 16, ...), kBlkRpg node rows
// per group with every load of the first pass issued before any use; the K
// values of (row i, block s) are contiguous.  The K * kBlkRpg sums leave a
// 16-lane reduction in lanes 0 .. K*kBlkRpg-1, which hold consecutive scalar
// rows (one contiguous store).  DOT: block partial of x[r] * y[r].
// EPI (multigrid smoothing, multigrid.hip): 0 y = A x; 1 y = x + omega dinv (b - A x); 2 y = b - A x.
constexpr int kBlkRpg = 2;
template <int K, bool DOT, int EPI = 0>
__global__ __launch_bounds__(256) void k_spmv_blk(int64_t n_brows, const int64_t* __restrict__ bp,
                                                  const int32_t* __restrict__ bc, const double* __restrict__ vals,
                                                  const double* __restrict__ x, double* __restrict__ y,
                                                  double* __restrict__ partial,
                                                  const int32_t* __restrict__ blist = nullptr,
                                                  const double* __restrict__ b = nullptr,
                                                  const double* __restrict__ dinv = nullptr, double omega = 0.0)
{
  const int l16 = threadIdx.x & 15;
  // blist: the row blocks of this launch (the CG's interior / halo-boundary split)
  const int64_t blk = blist ? (int64_t)blist[blockIdx.x] : xcd_swizzle(blockIdx.x, gridDim.x);
  const int64_t r0 = ((blk * 256 + threadIdx.x) >> 4) * kBlkRpg;
  int64_t b0[kBlkRpg];
  int len[kBlkRpg];
#pragma unroll
  for (int i = 0; i < kBlkRpg; ++i) {
    const int64_t r = r0 + i < n_brows ? r0 + i : n_brows - 1;
    b0[i] = bp[r];
    len[i] = r0 + i < n_brows ? (int)(bp[r + 1] - b0[i]) : 0;
  }
  double s[kBlkRpg][K];
  {
    int32_t c[kBlkRpg];
    double v[kBlkRpg][K][K];
#pragma unroll
    for (int i = 0; i < kBlkRpg; ++i) {
      const bool in = l16 < len[i];
      const int64_t kb = in ? b0[i] + l16 : b0[0];
      c[i] = in ? bc[kb] : 0;
      const double* vr = vals + (in ? K * K * b0[i] + K * l16 : 0);
#pragma unroll
      for (int a = 0; a < K; ++a)
#pragma unroll
        for (int j = 0; j < K; ++j) v[i][a][j] = in ? vr[K * a * len[i] + j] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < kBlkRpg; ++i) {
      double xv[K];
#pragma unroll
      for (int j = 0; j < K; ++j) xv[j] = x[K * (int64_t)c[i] + j];
#pragma unroll
      for (int a = 0; a < K; ++a) {
        double t = v[i][a][0] * xv[0];
#pragma unroll
        for (int j = 1; j < K; ++j) t = fma(v[i][a][j], xv[j], t);
        s[i][a] = t;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < kBlkRpg; ++i)
    for (int t = l16 + 16; t < len[i]; t += 16) {
      const int64_t cb = K * (int64_t)bc[b0[i] + t];
      const double* vr = vals + K * K * b0[i] + K * t;
#pragma unroll
      for (int a = 0; a < K; ++a) {
        double u = s[i][a];
#pragma unroll
        for (int j = 0; j < K; ++j) u = fma(vr[K * a * len[i] + j], x[cb + j], u);
        s[i][a] = u;
      }
    }
#pragma unroll
  for (int i = 0; i < kBlkRpg; ++i)
#pragma unroll
    for (int a = 0; a < K; ++a)
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) s[i][a] += __shfl_xor(s[i][a], o, 16);
  double d = 0.0;
  if (l16 < K * kBlkRpg) {
    double si = s[0][0];
#pragma unroll
    for (int q = 1; q < K * kBlkRpg; ++q)
      if (l16 == q) si = s[q / K][q % K];
    const int64_t r = K * r0 + l16;
    if (r < K * n_brows) {
      if constexpr (EPI == 1) y[r] = x[r] + omega * dinv[r] * (b[r] - si);
      else if constexpr (EPI == 2) y[r] = b[r] - si;
      else y[r] = si;
      if (DOT) d = x[r] * si;
    }
  }
  if (DOT) {
    double bs = block_sum(d);
    if (threadIdx.x == 0) partial[blockIdx.x] = bs;
  }
}

// The block-3 product on an fp32 copy of the values in a private layout
// (multigrid smoothing and residual on the fine level, AFEM_MG_F32): block q's
// row a is one 16-B word vf[4 (3 q + a) ..] = {v_a0, v_a1, v_a2, 0}, so a lane
// reads its block with three 16-B loads (the fp64 CSR order takes nine 8-B
// loads; a first fp32 version in the CSR order, nine 4-B loads per block, was
// slower than fp64 -- r05, the loads' count, not their bytes, set its rate).
// 52 instead of 76 B per block.  Same lanes, reduction and epilogues as
// k_spmv_blk<3, false, EPI>; products and sums in fp64.  EPI 3: the multigrid
// preconditioner's last sweep written straight into z with its constraint rows
// (z = x + omega dinv (b - A x), constraint rows rin dfix: mg_apply's copy and
// k_mg_fix folded in)
template <int EPI>
__global__ __launch_bounds__(256) void k_spmv_blk3f(int64_t n_brows, const int64_t* __restrict__ bp,
                                                    const int32_t* __restrict__ bc, const float4* __restrict__ vf,
                                                    const double* __restrict__ x, double* __restrict__ y,
                                                    const double* __restrict__ b, const double* __restrict__ dinv,
                                                    double omega, const uint8_t* __restrict__ cons = nullptr,
                                                    const double* __restrict__ rin = nullptr,
                                                    const double* __restrict__ dfix = nullptr)
{
  constexpr int K = 3;
  const int l16 = threadIdx.x & 15;
  const int64_t blk = xcd_swizzle(blockIdx.x, gridDim.x);
  const int64_t r0 = ((blk * 256 + threadIdx.x) >> 4) * kBlkRpg;
  int64_t b0[kBlkRpg];
  int len[kBlkRpg];
#pragma unroll
  for (int i = 0; i < kBlkRpg; ++i) {
    const int64_t r = r0 + i < n_brows ? r0 + i : n_brows - 1;
    b0[i] = bp[r];
    len[i] = r0 + i < n_brows ? (int)(bp[r + 1] - b0[i]) : 0;
  }
  double s[kBlkRpg][K];
  {
    int32_t c[kBlkRpg];
    float4 v[kBlkRpg][K];
#pragma unroll
    for (int i = 0; i < kBlkRpg; ++i) {
      const bool in = l16 < len[i];
      const int64_t q = in ? b0[i] + l16 : 0;
      c[i] = in ? bc[q] : 0;
#pragma unroll
      for (int a = 0; a < K; ++a) v[i][a] = vf[3 * q + a];
      if (!in) {
#pragma unroll
        for (int a = 0; a < K; ++a) v[i][a] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int i = 0; i < kBlkRpg; ++i) {
      double xv[K];
#pragma unroll
      for (int j = 0; j < K; ++j) xv[j] = x[K * (int64_t)c[i] + j];
#pragma unroll
      for (int a = 0; a < K; ++a) {
        double t = (double)v[i][a].x * xv[0];
        t = fma((double)v[i][a].y, xv[1], t);
        t = fma((double)v[i][a].z, xv[2], t);
        s[i][a] = t;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < kBlkRpg; ++i)
    for (int t = l16 + 16; t < len[i]; t += 16) {
      const int64_t q = b0[i] + t;
      const int64_t cb = K * (int64_t)bc[q];
#pragma unroll
      for (int a = 0; a < K; ++a) {
        const float4 w = vf[3 * q + a];
        double u = s[i][a];
        u = fma((double)w.x, x[cb], u);
        u = fma((double)w.y, x[cb + 1], u);
        u = fma((double)w.z, x[cb + 2], u);
        s[i][a] = u;
      }
    }
#pragma unroll
  for (int i = 0; i < kBlkRpg; ++i)
#pragma unroll
    for (int a = 0; a < K; ++a)
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) s[i][a] += __shfl_xor(s[i][a], o, 16);
  if (l16 < K * kBlkRpg) {
    double si = s[0][0];
#pragma unroll
    for (int q = 1; q < K * kBlkRpg; ++q)
      if (l16 == q) si = s[q / K][q % K];
    const int64_t r = K * r0 + l16;
    if (r < K * n_brows) {
      if constexpr (EPI == 1) y[r] = x[r] + omega * dinv[r] * (b[r] - si);
      else if constexpr (EPI == 3) y[r] = cons[r] ? rin[r] * dfix[r] : x[r] + omega * dinv[r] * (b[r] - si);
      else if constexpr (EPI == 2) y[r] = b[r] - si;
      else y[r] = si;
    }
  }
}

// fp32 saturated (a penalty beyond the fp32 range becomes its largest value, never inf: inf * 0 on a
// constraint row would be NaN)
__device__ __forceinline__ float f32_sat(double v)
{
  return (float)fmin(fmax(v, -3.4028234663852886e38), 3.4028234663852886e38);
}

// the private fp32 layout from BSRFormat's CSR order (16 lanes per node row, lane t:
// blocks t, t + 16, ...)
__global__ __launch_bounds__(256) void k_blk3_to_f32(int64_t n_brows, const int64_t* __restrict__ bp,
                                                     const double* __restrict__ vals, float4* __restrict__ vf)
{
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const int l16 = threadIdx.x & 15;
  if (r >= n_brows) return;
  const int64_t b0 = bp[r];
  const int len = (int)(bp[r + 1] - b0);
  for (int t = l16; t < len; t += 16) {
    const double* vr = vals + 9 * b0 + 3 * t;
#pragma unroll
    for (int a = 0; a < 3; ++a)
      vf[3 * (b0 + t) + a] = make_float4(f32_sat(vr[3 * a * len]), f32_sat(vr[3 * a * len + 1]),
                                         f32_sat(vr[3 * a * len + 2]), 0.f);
  }
}

// Fallback for segments that do not fit LDS: one lane per row.
template <bool DOT>
__global__ __launch_bounds__(kThreads) void k_spmv_row(int64_t n_rows, const int64_t* __restrict__ rows,
                                                       const int32_t* __restrict__ cols,
                                                       const double* __restrict__ vals, const double* __restrict__ x,
                                                       double* __restrict__ y, double* __restrict__ partial)
{
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double d = 0.0;
  if (r < n_rows) {
    double s = 0.0;
    for (int64_t k = rows[r]; k < rows[r + 1]; ++k) s += vals[k] * x[cols[k]];
    y[r] = s;
    if (DOT) d = x[r] * s;
  }
  if (DOT) {
    double bs = block_sum(d);
    if (threadIdx.x == 0) partial[blockIdx.x] = bs;
  }
}

__global__ __launch_bounds__(1024) void k_reduce(int64_t n, const double* __restrict__ partial,
                                                 double* __restrict__ out)
{
  __shared__ double ws[16];
  // 8 independent loads in flight per thread and round (a dependent load per
  // add made the reduce a latency chain: 11 us for the 39 k block partials of
  // C2), summed in a fixed order (deterministic)
  double s = 0.0;
  const int64_t step = blockDim.x;
  int64_t i = threadIdx.x;
  for (; i + 7 * step < n; i += 8 * step) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = partial[i + u * step];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; i < n; i += step) s += partial[i];
  s = wave_sum(s);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) ws[wid] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += ws[w];
    *out = t;
  }
}

// k_reduce over gridDim.x contiguous chunks of partial[0, n): chunk b's sum in out[b]
__global__ __launch_bounds__(1024) void k_reduce_chunks(int64_t n, const double* __restrict__ partial,
                                                        double* __restrict__ out)
{
  __shared__ double ws[16];
  const int64_t c0 = n * blockIdx.x / gridDim.x, c1 = n * (blockIdx.x + 1) / gridDim.x;
  double s = 0.0;
  const int64_t step = blockDim.x;
  int64_t i = c0 + threadIdx.x;
  for (; i + 7 * step < c1; i += 8 * step) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = partial[i + u * step];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; i < c1; i += step) s += partial[i];
  s = wave_sum(s);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) ws[wid] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += ws[w];
    out[blockIdx.x] = t;
  }
}

// Jacobi preconditioner + constraint-row flag: a row whose diagonal exceeds
// the rest of the row by > 1e10 (penalty P = 1e30, eliminated identity rows)
// is excluded from the reference value of the stopping test (same rule as
// oracle/oracle.c::orc_pcg_jacobi; duplicate (i,i) entries of a view add up,
// as the SpMV applies them).
// 16 lanes per row: the row's columns and values are read coalesced (one
// thread per row walked 15 entries 120 B apart from its neighbours': 20 ms per
// solve at C4), the diagonal and the |off-diagonal| sum are 16-lane
// reductions; a grid-stride loop over rows (one wave per 4 rows: 25 M waves
// at C4, 7 ms, the launch of that many waves rather than the 18 GB read)
__global__ __launch_bounds__(256) void k_inv_diag(int64_t n_rows, const int64_t* __restrict__ rows,
                                                  const int32_t* __restrict__ cols, const double* __restrict__ vals,
                                                  double* __restrict__ dinv, uint8_t* __restrict__ cons)
{
  const int l16 = threadIdx.x & 15;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x / 16;
  for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4; r < n_rows; r += stride) {
    const int64_t a = rows[r], e = rows[r + 1];
    double d = 0.0, off = 0.0;
    for (int64_t k = a + l16; k < e; k += 16) {
      const double v = vals[k];
      if (cols[k] == (int32_t)r)
        d += v;
      else
        off += fabs(v);
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      d += __shfl_xor(d, o, 16);
      off += __shfl_xor(off, o, 16);
    }
    if (l16 == 0) {
      dinv[r] = (d != 0.0) ? 1.0 / d : 0.0;
      cons[r] = fabs(d) > 1e10 * off ? 1 : 0;
    }
  }
}

// k_inv_diag for a system with a node-block structure (NB_DOF = K, BSRFormat's
// CSR order): 16 lanes per node row read its K x K blocks coalesced (one
// thread per scalar row walks 45 scattered values on a block-3 system: 10 ms
// per solve at C5 size), the diagonal and the |off-diagonal| sums of the K
// scalar rows are 16-lane reductions.
template <int K>
__global__ __launch_bounds__(256) void k_inv_diag_blk(int64_t n_brows, const int64_t* __restrict__ bp,
                                                      const int32_t* __restrict__ bc,
                                                      const double* __restrict__ vals, double* __restrict__ dinv,
                                                      uint8_t* __restrict__ cons)
{
  const int l16 = threadIdx.x & 15;
  const int64_t r = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
  const int64_t rr = r < n_brows ? r : n_brows - 1;
  const int64_t b0 = bp[rr];
  const int len = (int)(bp[rr + 1] - b0);
  double d[K], off[K];
#pragma unroll
  for (int a = 0; a < K; ++a) d[a] = off[a] = 0.0;
  for (int t = l16; t < len; t += 16) {
    const bool diag = bc[b0 + t] == (int32_t)rr;
    const double* v = vals + K * K * b0 + K * t;
#pragma unroll
    for (int a = 0; a < K; ++a)
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const double x = v[K * a * len + j];
        if (diag && j == a) d[a] = x;
        else off[a] += fabs(x);
      }
  }
#pragma unroll
  for (int a = 0; a < K; ++a)
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      d[a] += __shfl_xor(d[a], o, 16);
      off[a] += __shfl_xor(off[a], o, 16);
    }
  if (l16 < K && r < n_brows) {
    double da = d[0], oa = off[0];
#pragma unroll
    for (int a = 1; a < K; ++a)
      if (l16 == a) {
        da = d[a];
        oa = off[a];
      }
    dinv[K * r + l16] = (da != 0.0) ? 1.0 / da : 0.0;
    cons[K * r + l16] = fabs(da) > 1e10 * oa ? 1 : 0;
  }
}

constexpr int kVecBlocks = 2048;

// Initial guess: constraint rows solved on their own (x0_i = b_i / a_ii: the
// Dirichlet value for penalty and eliminated rows), 0 elsewhere.  This lifts
// the Dirichlet data into x0, so the residual of the free rows carries it
// from the start (the stopping reference is then meaningful also for
// problems driven only by Dirichlet data), and the eliminated rows keep a
// zero residual and search direction, so a row-eliminated (non-symmetric)
// system is iterated on its symmetric free block.
__global__ __launch_bounds__(kThreads) void k_cg_x0(int64_t n, const double* __restrict__ b,
                                                    const double* __restrict__ dinv, const uint8_t* __restrict__ cons,
                                                    double* __restrict__ x, double* __restrict__ p)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double xi = cons[i] ? b[i] * dinv[i] : 0.0;
    x[i] = xi;
    p[i] = xi;
  }
}

// Initial guess from the caller (afem_solver_opts::initial_guess = 1): the
// constraint rows lifted as in k_cg_x0, the free rows from g
__global__ __launch_bounds__(kThreads) void k_cg_x0_guess(int64_t n, const double* __restrict__ b,
                                                          const double* __restrict__ dinv,
                                                          const uint8_t* __restrict__ cons,
                                                          const double* __restrict__ g, double* __restrict__ x,
                                                          double* __restrict__ p)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double xi = cons[i] ? b[i] * dinv[i] : g[i];
    x[i] = xi;
    p[i] = xi;
  }
}

// r = b - A x0 (q), z = D^-1 r, p = z ; partials r.z (all rows) and r.z (free rows)
__global__ __launch_bounds__(kThreads) void k_cg_init(int64_t n, const double* __restrict__ b,
                                                      const double* __restrict__ q, double* __restrict__ r,
                                                      double* __restrict__ z, double* __restrict__ p,
                                                      const double* __restrict__ dinv,
                                                      const uint8_t* __restrict__ cons, double* __restrict__ partial,
                                                      double* __restrict__ partial_free)
{
  double s = 0.0, sf = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double ri = b[i] - q[i];
    double zi = ri * dinv[i];
    r[i] = ri;
    z[i] = zi;
    p[i] = zi;
    s += ri * zi;
    if (!cons[i]) sf += ri * zi;
  }
  double bs = block_sum(s);
  double bf = block_sum(sf);
  if (threadIdx.x == 0) {
    partial[blockIdx.x] = bs;
    partial_free[blockIdx.x] = bf;
  }
}

// ---- block-Jacobi (3x3 node blocks, afem_solver_opts::precond_block = 3:
// the NB_DOF = 3 systems of elasticity / elastodynamics).  The block of node
// b is rows/cols 3b..3b+2 of the CSR; a constraint row (penalty / eliminated,
// `cons`) is decoupled from its block mates before the inversion, so the
// preconditioner is block-diag(1/a_ii, inverse of the free sub-block): SPD
// when the free block is, and the constraint rows keep z_i = r_i / a_ii.
__global__ void k_inv_block3(int64_t nb, const int64_t* __restrict__ rows, const int32_t* __restrict__ cols,
                             const double* __restrict__ vals, const uint8_t* __restrict__ cons,
                             const double* __restrict__ dinv, double* __restrict__ binv)
{
  const int64_t ib = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ib >= nb) return;
  double B[3][3] = { { 0, 0, 0 }, { 0, 0, 0 }, { 0, 0, 0 } };
  bool c[3];
  for (int a = 0; a < 3; ++a) {
    const int64_t row = 3 * ib + a;
    c[a] = cons[row] != 0;
    for (int64_t k = rows[row]; k < rows[row + 1]; ++k) {
      const int64_t d = (int64_t)cols[k] - 3 * ib;
      if (d >= 0 && d < 3) B[a][d] = vals[k];
    }
  }
  for (int a = 0; a < 3; ++a)
    for (int d = 0; d < 3; ++d)
      if (a != d && (c[a] || c[d])) B[a][d] = 0.0;
  const double c00 = B[1][1] * B[2][2] - B[1][2] * B[2][1], c01 = B[1][2] * B[2][0] - B[1][0] * B[2][2],
               c02 = B[1][0] * B[2][1] - B[1][1] * B[2][0];
  const double det = B[0][0] * c00 + B[0][1] * c01 + B[0][2] * c02;
  double* o = binv + 9 * ib;
  if (det == 0.0 || !isfinite(det)) {  // singular block: point Jacobi
    for (int a = 0; a < 3; ++a)
      for (int d = 0; d < 3; ++d) o[3 * a + d] = a == d ? dinv[3 * ib + a] : 0.0;
    return;
  }
  const double id = 1.0 / det;
  o[0] = c00 * id;
  o[1] = (B[0][2] * B[2][1] - B[0][1] * B[2][2]) * id;
  o[2] = (B[0][1] * B[1][2] - B[0][2] * B[1][1]) * id;
  o[3] = c01 * id;
  o[4] = (B[0][0] * B[2][2] - B[0][2] * B[2][0]) * id;
  o[5] = (B[0][2] * B[1][0] - B[0][0] * B[1][2]) * id;
  o[6] = c02 * id;
  o[7] = (B[0][1] * B[2][0] - B[0][0] * B[2][1]) * id;
  o[8] = (B[0][0] * B[1][1] - B[0][1] * B[1][0]) * id;
}

__device__ __forceinline__ void apply_binv3(const double* __restrict__ m, const double (&r)[3], double (&z)[3])
{
  z[0] = m[0] * r[0] + m[1] * r[1] + m[2] * r[2];
  z[1] = m[3] * r[0] + m[4] * r[1] + m[5] * r[2];
  z[2] = m[6] * r[0] + m[7] * r[1] + m[8] * r[2];
}

// k_cg_init with z = Binv r per node block (nb = n / 3 blocks)
__global__ __launch_bounds__(kThreads) void k_cg_init_b3(int64_t nb, const double* __restrict__ b,
                                                         const double* __restrict__ q, double* __restrict__ r,
                                                         double* __restrict__ z, double* __restrict__ p,
                                                         const double* __restrict__ binv,
                                                         const uint8_t* __restrict__ cons, double* __restrict__ partial,
                                                         double* __restrict__ partial_free)
{
  double s = 0.0, sf = 0.0;
  for (int64_t ib = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; ib < nb; ib += (int64_t)gridDim.x * blockDim.x) {
    double ri[3], zi[3];
    for (int a = 0; a < 3; ++a) ri[a] = b[3 * ib + a] - q[3 * ib + a];
    apply_binv3(binv + 9 * ib, ri, zi);
    for (int a = 0; a < 3; ++a) {
      r[3 * ib + a] = ri[a];
      z[3 * ib + a] = zi[a];
      p[3 * ib + a] = zi[a];
      s += ri[a] * zi[a];
      if (!cons[3 * ib + a]) sf += ri[a] * zi[a];
    }
  }
  double bs = block_sum(s);
  double bf = block_sum(sf);
  if (threadIdx.x == 0) {
    partial[blockIdx.x] = bs;
    partial_free[blockIdx.x] = bf;
  }
}

// k_cg_update with z = Binv r per node block
__global__ __launch_bounds__(kThreads) void k_cg_update_b3(int64_t nb, const double* __restrict__ scal, int par,
                                                           double* __restrict__ x, const double* __restrict__ p,
                                                           double* __restrict__ r, const double* __restrict__ q,
                                                           double* __restrict__ z, const double* __restrict__ binv,
                                                           double* __restrict__ partial)
{
  const double rz = scal[par], pq = scal[2];
  const double alpha = (pq != 0.0) ? rz / pq : 0.0;
  double s = 0.0;
  for (int64_t ib = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; ib < nb; ib += (int64_t)gridDim.x * blockDim.x) {
    double ri[3], zi[3];
    for (int a = 0; a < 3; ++a) {
      x[3 * ib + a] += alpha * p[3 * ib + a];
      ri[a] = r[3 * ib + a] - alpha * q[3 * ib + a];
      r[3 * ib + a] = ri[a];
    }
    apply_binv3(binv + 9 * ib, ri, zi);
    for (int a = 0; a < 3; ++a) {
      z[3 * ib + a] = zi[a];
      s += ri[a] * zi[a];
    }
  }
  double bs = block_sum(s);
  if (threadIdx.x == 0) partial[blockIdx.x] = bs;
}

// The point-Jacobi iteration's vector pass split so that no vector is read
// twice: k_cg_update_rz (r, z and the partial r.z: reads r, q, dinv, writes
// r, z) and k_cg_dir_x (x += alpha p with the p of this iteration, then
// p = z + beta p: reads x, z, p, writes x, p) -- 80 B per row instead of the
// 88 of k_cg_update + k_cg_dir; the same operations on the same values.
// V2: two rows per thread and access (16-B loads / stores per lane)
// V2: 16-B accesses (two rows per access); U2 (with V2): two such accesses per
// thread and iteration, [i] and [i + stride] (more loads in flight)
template <bool V2, bool U2 = false>
__global__ __launch_bounds__(kThreads) void k_cg_update_rz(int64_t n, const double* __restrict__ scal, int par,
                                                           double* __restrict__ r, const double* __restrict__ q,
                                                           double* __restrict__ z, const double* __restrict__ dinv,
                                                           double* __restrict__ partial)
{
  const double rz = scal[par], pq = scal[2];
  const double alpha = (pq != 0.0) ? rz / pq : 0.0;
  double s = 0.0;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t)gridDim.x * blockDim.x;
  if constexpr (V2 && U2) {
    double2* r2 = reinterpret_cast<double2*>(r);
    double2* z2 = reinterpret_cast<double2*>(z);
    const double2* q2 = reinterpret_cast<const double2*>(q);
    const double2* d2 = reinterpret_cast<const double2*>(dinv);
    const int64_t m = n >> 1;
    for (int64_t i = t0; i < m; i += 2 * st) {
      const bool two = i + st < m;
      double2 ra = r2[i], rb = two ? r2[i + st] : make_double2(0.0, 0.0);
      const double2 qa = q2[i], qb = two ? q2[i + st] : make_double2(0.0, 0.0);
      const double2 da = d2[i], db = two ? d2[i + st] : make_double2(0.0, 0.0);
      ra.x = ra.x - alpha * qa.x;
      ra.y = ra.y - alpha * qa.y;
      rb.x = rb.x - alpha * qb.x;
      rb.y = rb.y - alpha * qb.y;
      const double2 za = make_double2(ra.x * da.x, ra.y * da.y), zb = make_double2(rb.x * db.x, rb.y * db.y);
      r2[i] = ra;
      z2[i] = za;
      if (two) {
        r2[i + st] = rb;
        z2[i + st] = zb;
      }
      s += ra.x * za.x;
      s += ra.y * za.y;
      s += rb.x * zb.x;
      s += rb.y * zb.y;
    }
    if ((n & 1) && t0 == 0) {
      const int64_t i = n - 1;
      double ri = r[i] - alpha * q[i];
      r[i] = ri;
      double zi = ri * dinv[i];
      z[i] = zi;
      s += ri * zi;
    }
  }
  else if constexpr (V2) {
    double2* r2 = reinterpret_cast<double2*>(r);
    double2* z2 = reinterpret_cast<double2*>(z);
    const double2* q2 = reinterpret_cast<const double2*>(q);
    const double2* d2 = reinterpret_cast<const double2*>(dinv);
    for (int64_t i = t0; i < (n >> 1); i += st) {
      double2 rv = r2[i];
      const double2 qv = q2[i], dv = d2[i];
      rv.x = rv.x - alpha * qv.x;
      rv.y = rv.y - alpha * qv.y;
      r2[i] = rv;
      const double2 zv = make_double2(rv.x * dv.x, rv.y * dv.y);
      z2[i] = zv;
      s += rv.x * zv.x;
      s += rv.y * zv.y;
    }
    if ((n & 1) && t0 == 0) {
      const int64_t i = n - 1;
      double ri = r[i] - alpha * q[i];
      r[i] = ri;
      double zi = ri * dinv[i];
      z[i] = zi;
      s += ri * zi;
    }
  }
  else {
    for (int64_t i = t0; i < n; i += st) {
      double ri = r[i] - alpha * q[i];
      r[i] = ri;
      double zi = ri * dinv[i];
      z[i] = zi;
      s += ri * zi;
    }
  }
  double bs = block_sum(s);
  if (threadIdx.x == 0) partial[blockIdx.x] = bs;
}
template <bool V2, bool U2 = false>
__global__ __launch_bounds__(kThreads) void k_cg_dir_x(int64_t n, const double* __restrict__ scal, int par,
                                                       double* __restrict__ x, const double* __restrict__ z,
                                                       double* __restrict__ p)
{
  const double rz_old = scal[par], rz_new = scal[par ^ 1], pq = scal[2];
  const double alpha = (pq != 0.0) ? rz_old / pq : 0.0;
  const double beta = (rz_old != 0.0) ? rz_new / rz_old : 0.0;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t)gridDim.x * blockDim.x;
  if constexpr (V2 && U2) {
    double2* x2 = reinterpret_cast<double2*>(x);
    double2* p2 = reinterpret_cast<double2*>(p);
    const double2* z2 = reinterpret_cast<const double2*>(z);
    const int64_t m = n >> 1;
    for (int64_t i = t0; i < m; i += 2 * st) {
      const bool two = i + st < m;
      const double2 pa = p2[i], za = z2[i];
      double2 xa = x2[i];
      const double2 pb = two ? p2[i + st] : make_double2(0.0, 0.0), zb = two ? z2[i + st] : make_double2(0.0, 0.0);
      double2 xb = two ? x2[i + st] : make_double2(0.0, 0.0);
      xa.x += alpha * pa.x;
      xa.y += alpha * pa.y;
      xb.x += alpha * pb.x;
      xb.y += alpha * pb.y;
      x2[i] = xa;
      p2[i] = make_double2(za.x + beta * pa.x, za.y + beta * pa.y);
      if (two) {
        x2[i + st] = xb;
        p2[i + st] = make_double2(zb.x + beta * pb.x, zb.y + beta * pb.y);
      }
    }
    if ((n & 1) && t0 == 0) {
      const int64_t i = n - 1;
      const double pi = p[i];
      x[i] += alpha * pi;
      p[i] = z[i] + beta * pi;
    }
  }
  else if constexpr (V2) {
    double2* x2 = reinterpret_cast<double2*>(x);
    double2* p2 = reinterpret_cast<double2*>(p);
    const double2* z2 = reinterpret_cast<const double2*>(z);
    for (int64_t i = t0; i < (n >> 1); i += st) {
      const double2 pv = p2[i], zv = z2[i];
      double2 xv = x2[i];
      xv.x += alpha * pv.x;
      xv.y += alpha * pv.y;
      x2[i] = xv;
      p2[i] = make_double2(zv.x + beta * pv.x, zv.y + beta * pv.y);
    }
    if ((n & 1) && t0 == 0) {
      const int64_t i = n - 1;
      const double pi = p[i];
      x[i] += alpha * pi;
      p[i] = z[i] + beta * pi;
    }
  }
  else {
    for (int64_t i = t0; i < n; i += st) {
      const double pi = p[i];
      x[i] += alpha * pi;
      p[i] = z[i] + beta * pi;
    }
  }
}

// beta = rz_new / rz_old ; p = z + beta p
// x += alpha p, r -= alpha q (the multigrid-preconditioned PCG forms z separately)
__global__ __launch_bounds__(kThreads) void k_cg_xr(int64_t n, const double* __restrict__ scal, int par,
                                                    double* __restrict__ x, const double* __restrict__ p,
                                                    double* __restrict__ r, const double* __restrict__ q)
{
  const double rz = scal[par], pq = scal[2];
  const double alpha = (pq != 0.0) ? rz / pq : 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    x[i] += alpha * p[i];
    r[i] -= alpha * q[i];
  }
}

__global__ __launch_bounds__(kThreads) void k_cg_dir(int64_t n, const double* __restrict__ scal, int par,
                                                     const double* __restrict__ z, double* __restrict__ p)
{
  const double rz_old = scal[par], rz_new = scal[par ^ 1];
  const double beta = (rz_old != 0.0) ? rz_new / rz_old : 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = z[i] + beta * p[i];
}

// flexible CG (Polak-Ribiere; Notay's FCG(1)) for a nonlinear preconditioner
// (the AMG K-cycle): beta = z_new.(r_new - r_old) / rz_old = -(z_new.q) / (p.q),
// since r_new - r_old = -alpha q and alpha = rz_old / (p.q); scal[5] = z_new.q
__global__ __launch_bounds__(kThreads) void k_cg_dir_flex(int64_t n, const double* __restrict__ scal,
                                                          const double* __restrict__ z, double* __restrict__ p)
{
  const double pq = scal[2], zq = scal[5];
  const double beta = (pq != 0.0) ? -zq / pq : 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = z[i] + beta * p[i];
}

__global__ __launch_bounds__(kThreads) void k_dot(int64_t n, const double* __restrict__ a,
                                                  const double* __restrict__ b, double* __restrict__ partial)
{
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    s += a[i] * b[i];
  double bs = block_sum(s);
  if (threadIdx.x == 0) partial[blockIdx.x] = bs;
}

// ---------------------------------------------------------------- direct solver
// The direct branch of SequentialDoFLinearSystemImpl::solve (N < 500,
// femutils/DoFLinearSystem.cc:127-136; Arcane MatVec::DirectSolver is external,
// so its pivoting is unpinned): dense Gaussian elimination with partial
// pivoting on the augmented n x (n+1) matrix [A | b], row-major in HBM, by
// one 1024-lane workgroup (n <= 4096: at most 128 MiB and a few ms), then
// column-oriented back substitution.  Ghost columns (>= n) are dropped: on
// one rank their values are not unknowns of this system.
constexpr int kDirectThreads = 1024;

__global__ void k_csr_to_dense(int64_t n, const int64_t* __restrict__ rows, const int32_t* __restrict__ cols,
                               const double* __restrict__ vals, const double* __restrict__ b, double* __restrict__ a)
{
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  double* ar = a + r * (n + 1);
  for (int64_t j = 0; j <= n; ++j) ar[j] = 0.0;
  for (int64_t k = rows[r]; k < rows[r + 1]; ++k)
    if (cols[k] < n) ar[cols[k]] += vals[k];
  ar[n] = b[r];
}

__global__ __launch_bounds__(kDirectThreads) void k_dense_gauss(int n, double* __restrict__ a, double* __restrict__ x,
                                                                int* __restrict__ singular)
{
  __shared__ double sv[kDirectThreads / 64];
  __shared__ int si[kDirectThreads / 64];
  __shared__ int piv;
  const int ld = n + 1, t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) *singular = 0;
  for (int k = 0; k < n; ++k) {
    // pivot: argmax_i>=k |a_ik| (lowest row index on ties)
    double bv = -1.0;
    int bi = k;
    for (int i = k + t; i < n; i += kDirectThreads) {
      const double v = fabs(a[(int64_t)i * ld + k]);
      if (v > bv) {
        bv = v;
        bi = i;
      }
    }
    for (int d = 32; d > 0; d >>= 1) {
      const double ov = __shfl_xor(bv, d, 64);
      const int oi = __shfl_xor(bi, d, 64);
      if (ov > bv || (ov == bv && oi < bi)) {
        bv = ov;
        bi = oi;
      }
    }
    if (lane == 0) {
      sv[w] = bv;
      si[w] = bi;
    }
    __syncthreads();
    if (t == 0) {
      double v = sv[0];
      int i0 = si[0];
      for (int q = 1; q < kDirectThreads / 64; ++q)
        if (sv[q] > v || (sv[q] == v && si[q] < i0)) {
          v = sv[q];
          i0 = si[q];
        }
      piv = i0;
      if (!(v > 0.0)) *singular = 1;
    }
    __syncthreads();
    const int p = piv;
    if (p != k)
      for (int j = k + t; j <= n; j += kDirectThreads) {
        const double tmp = a[(int64_t)k * ld + j];
        a[(int64_t)k * ld + j] = a[(int64_t)p * ld + j];
        a[(int64_t)p * ld + j] = tmp;
      }
    __syncthreads();
    const double inv = 1.0 / a[(int64_t)k * ld + k];
    const int wdt = n - k;  // columns k+1..n
    const int64_t tot = (int64_t)(n - k - 1) * wdt;
    for (int64_t e = t; e < tot; e += kDirectThreads) {
      const int i = k + 1 + (int)(e / wdt), j = k + 1 + (int)(e % wdt);
      const double l = a[(int64_t)i * ld + k] * inv;
      a[(int64_t)i * ld + j] -= l * a[(int64_t)k * ld + j];
    }
    __syncthreads();
  }
  // back substitution, column oriented: x_j = c_j / u_jj, c_i -= u_ij x_j (i < j)
  for (int j = n - 1; j >= 0; --j) {
    const double xj = a[(int64_t)j * ld + n] / a[(int64_t)j * ld + j];
    for (int i = t; i < j; i += kDirectThreads) a[(int64_t)i * ld + n] -= a[(int64_t)i * ld + j] * xj;
    if (t == 0) x[j] = xj;
    __syncthreads();
  }
}

// r = b - A x (owned rows), partial sums of r.r and b.b
__global__ __launch_bounds__(256) void k_residual(int64_t n, const int64_t* __restrict__ rows,
                                                  const int32_t* __restrict__ cols, const double* __restrict__ vals,
                                                  const double* __restrict__ x, const double* __restrict__ b,
                                                  double* __restrict__ partial)
{
  double rr = 0.0, bb = 0.0;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int64_t k = rows[r]; k < rows[r + 1]; ++k)
      if (cols[k] < n) s += vals[k] * x[cols[k]];
    const double ri = b[r] - s;
    rr += ri * ri;
    bb += b[r] * b[r];
  }
  const double a = block_sum(rr);
  const double c = block_sum(bb);
  if (threadIdx.x == 0) {
    partial[2 * blockIdx.x] = a;
    partial[2 * blockIdx.x + 1] = c;
  }
}

// ---------------------------------------------------------------- helpers
// 1 if a row block reads a ghost column (col >= n_rows): its SpMV must wait
// for the halo exchange
__global__ __launch_bounds__(256) void k_block_ghost(int64_t n_rows, int rpb, const int64_t* __restrict__ rows,
                                                     const int32_t* __restrict__ cols, uint8_t* __restrict__ flag)
{
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = r0 + rpb < n_rows ? r0 + rpb : n_rows;
  int g = 0;
  for (int64_t k = rows[r0] + threadIdx.x; k < rows[r1]; k += blockDim.x) g |= cols[k] >= n_rows ? 1 : 0;
  g = __syncthreads_or(g);
  if (threadIdx.x == 0) flag[blockIdx.x] = (uint8_t)g;
}

struct SpmvPlan {
  int rpb = 0;          // rows per block (0: row kernel, -1: vector CSR, -2: node blocks)
  bool wide = false;    // 16-B loads of the segment (aligned bases)
  bool unroll = false;  // k_spmv_stream4u
  int64_t max_seg = 0;
  int64_t nblocks = 0;
  // rpb = -2: k_spmv_blk over the node-row structure (NB_DOF = blk_k)
  int blk_k = 0;
  int64_t blk_n = 0;
  const int64_t* blk_rows = nullptr;
  const int32_t* blk_cols = nullptr;
  // rpb = -3: k_spmv_pat (pattern rows form their columns), rows per block bs
  const uint8_t* pat_flag = nullptr;
  PatOff po{};
  int bs = kThreads;
};

__global__ void k_block_seg(int64_t n_rows, int rpb, const int64_t* __restrict__ row_ptr, unsigned long long* out)
{
  int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t r0 = b * rpb;
  if (r0 >= n_rows) return;
  int64_t r1 = r0 + rpb < n_rows ? r0 + rpb : n_rows;
  atomicMax(out, (unsigned long long)(row_ptr[r1] - row_ptr[r0]));
}

SpmvPlan plan_spmv(Ctx& ctx, const int64_t* rows, int64_t n_rows, const int32_t* cols = nullptr,
                   const double* vals = nullptr)
{
  SpmvPlan pl;
  DevBuf<unsigned long long> mx;
  mx.alloc(1);
  AFEM_HIP(hipMemsetAsync(mx.p, 0, mx.bytes(), ctx.stream));
  int64_t nb = (n_rows + kThreads - 1) / kThreads;
  hipLaunchKernelGGL(k_block_seg, dim3(grid_for(nb, 256)), dim3(256), 0, ctx.stream, n_rows, kThreads, rows, mx.p);
  AFEM_LAUNCHED();
  unsigned long long hm = 0;
  AFEM_HIP(hipMemcpyAsync(&hm, mx.p, sizeof(hm), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  pl.nblocks = nb;
  // AFEM_SPMV=stream (scalar-load stream) / v16 (16 lanes per row) / s4 (no unrolling): diagnostics
  const int mode = [] {  // read per plan (tools/cg_probe.py toggles it in one process)
    const char* e = variant("AFEM_SPMV");
    if (e && std::string(e) == "stream") return 1;
    if (e && std::string(e) == "v16") return 2;
    if (e && std::string(e) == "s4") return 3;
    return 0;
  }();
  if (mode == 2) {
    pl.rpb = -1;
    pl.nblocks = (n_rows + 16 * kSpmvRpg - 1) / (16 * kSpmvRpg);
  }
  else if (hm * 8ull <= 64ull * 1024ull) {
    pl.rpb = kThreads;
    pl.max_seg = (int64_t)hm;
    pl.wide = (mode == 0 || mode == 3) && cols && vals && ((uintptr_t)cols & 15) == 0 && ((uintptr_t)vals & 15) == 0;
    pl.unroll = mode == 0;
    // AFEM_SPMV_STREAM_BS=64 / 128: the unrolled stream kernel in smaller row blocks (its segment
    // bound and block count for that size).  Not the default: unlike the pattern kernel (no column-image
    // phase to overlap) it measured slower, C2 with the stream kernel 0.603 vs 0.597 ms per CG iteration,
    // the unstructured system's Jacobi-PCG 0.812 vs 0.795-0.799 (r05ao)
    const char* be = variant("AFEM_SPMV_STREAM_BS");
    const int bsz = be ? atoi(be) : kThreads;
    if (pl.unroll && pl.wide && (bsz == 64 || bsz == 128)) {
      AFEM_HIP(hipMemsetAsync(mx.p, 0, mx.bytes(), ctx.stream));
      const int64_t nbs = (n_rows + bsz - 1) / bsz;
      hipLaunchKernelGGL(k_block_seg, dim3(grid_for(nbs, 256)), dim3(256), 0, ctx.stream, n_rows, bsz, rows, mx.p);
      AFEM_LAUNCHED();
      unsigned long long hs = 0;
      AFEM_HIP(hipMemcpyAsync(&hs, mx.p, sizeof(hs), hipMemcpyDeviceToHost, ctx.stream));
      ctx.sync();
      pl.bs = bsz;
      pl.max_seg = (int64_t)hs;
      pl.nblocks = nbs;
    }
  }
  else if (mode == 0 && hm >= 16ull * (unsigned long long)kThreads) {
    // long rows (block-3 elasticity: 45 non-zeros per scalar row): segments do
    // not fit LDS; 16 lanes per row keep the column/value reads coalesced
    pl.rpb = -1;
    pl.nblocks = (n_rows + 16 * kSpmvRpg - 1) / (16 * kSpmvRpg);
  }
  return pl;
}

}  // namespace

void spmv_blk3f_epi(Ctx& ctx, int epi, int64_t n_brows, const int64_t* bp, const int32_t* bc, const float* vf,
                    const double* x, double* y, const double* b, const double* dinv, double omega,
                    const uint8_t* cons, const double* rin, const double* dfix)
{
  const unsigned nb = (unsigned)((n_brows + 16 * kBlkRpg - 1) / (16 * kBlkRpg));
  if (nb == 0) return;
  const float4* v4 = reinterpret_cast<const float4*>(vf);
  if (epi == 3)
    hipLaunchKernelGGL(k_spmv_blk3f<3>, dim3(nb), dim3(256), 0, ctx.stream, n_brows, bp, bc, v4, x, y, b, dinv, omega,
                       cons, rin, dfix);
  else if (epi == 1)
    hipLaunchKernelGGL(k_spmv_blk3f<1>, dim3(nb), dim3(256), 0, ctx.stream, n_brows, bp, bc, v4, x, y, b, dinv, omega);
  else if (epi == 2)
    hipLaunchKernelGGL(k_spmv_blk3f<2>, dim3(nb), dim3(256), 0, ctx.stream, n_brows, bp, bc, v4, x, y, b, dinv, omega);
  else
    hipLaunchKernelGGL(k_spmv_blk3f<0>, dim3(nb), dim3(256), 0, ctx.stream, n_brows, bp, bc, v4, x, y, b, dinv, omega);
  AFEM_LAUNCHED();
}

void blk3_to_f32(Ctx& ctx, int64_t n_brows, const int64_t* bp, const double* vals, float* vf)
{
  if (n_brows <= 0) return;
  hipLaunchKernelGGL(k_blk3_to_f32, dim3(grid_for(n_brows * 16, 256)), dim3(256), 0, ctx.stream, n_brows, bp, vals,
                     reinterpret_cast<float4*>(vf));
  AFEM_LAUNCHED();
}

void spmv_blk_epi(Ctx& ctx, int k, int epi, int64_t n_brows, const int64_t* bp, const int32_t* bc, const double* vals,
                  const double* x, double* y, const double* b, const double* dinv, double omega)
{
  const unsigned nb = (unsigned)((n_brows + 16 * kBlkRpg - 1) / (16 * kBlkRpg));
  if (nb == 0) return;
#define AFEM_EPI(K_, E_)                                                                                           \
  hipLaunchKernelGGL((k_spmv_blk<K_, false, E_>), dim3(nb), dim3(256), 0, ctx.stream, n_brows, bp, bc, vals, x, y, \
                     nullptr, nullptr, b, dinv, omega)
#define AFEM_EPI_K(K_)       \
  if (epi == 1)              \
    AFEM_EPI(K_, 1);         \
  else if (epi == 2)         \
    AFEM_EPI(K_, 2);         \
  else                       \
    AFEM_EPI(K_, 0);
  if (k == 3) {
    AFEM_EPI_K(3)
  }
  else if (k == 2) {
    AFEM_EPI_K(2)
  }
  else {
    AFEM_EPI_K(1)
  }
#undef AFEM_EPI_K
#undef AFEM_EPI
  AFEM_LAUNCHED();
}

namespace {

// the node-block SpMV when the system came from a BSRFormat with NB_DOF 2 or 3
// (AFEM_SPMV=csr or any other diagnostic mode keeps the scalar CSR kernels)
SpmvPlan plan_spmv_ls(Ctx& ctx, const LinearSystem& ls)
{
  SpmvPlan pl = plan_spmv(ctx, ls.csr_rows, ls.n_rows, ls.csr_cols, ls.csr_vals);
  const char* e = variant("AFEM_SPMV");
  // the pattern SpMV: the default for scalar systems (AFEM_SPMV=nopat or any other
  // diagnostic mode: the CSR kernels as they are)
  if ((!e || std::string(e) == "pat") && ls.blk_k <= 1 && ls.n_rows > 64 && ls.csr_cols && ls.csr_vals &&
      pl.rpb == kThreads && pl.wide && pl.max_seg + 3 <= 4 * kThreads * kSpmvU) {
    // the most frequent column-offset pattern among 256 rows spread over the
    // range (a structured box's interior stencil); rows that share it (k_pat_flags)
    constexpr int kSamples = 256;
    if (ls.pat_smp.n < (size_t)(kSamples * 17)) ls.pat_smp.alloc(kSamples * 17);
    hipLaunchKernelGGL(k_pat_sample, dim3(1), dim3(kSamples), 0, ctx.stream, ls.n_rows, ls.csr_rows, ls.csr_cols,
                       ls.pat_smp.p);
    AFEM_LAUNCHED();
    std::vector<int32_t> hs(kSamples * 17);
    AFEM_HIP(hipMemcpyAsync(hs.data(), ls.pat_smp.p, hs.size() * sizeof(int32_t), hipMemcpyDeviceToHost, ctx.stream));
    ctx.sync();
    std::map<std::vector<int64_t>, int> freq;
    for (int i = 0; i < kSamples; ++i) {
      const int len = hs[17 * i];
      if (len < 1 || len > 16) continue;
      ++freq[std::vector<int64_t>(hs.begin() + 17 * i + 1, hs.begin() + 17 * i + 1 + len)];
    }
    const std::vector<int64_t>* best = nullptr;
    int bc = 0;
    for (const auto& kv : freq)
      if (kv.second > bc) {
        bc = kv.second;
        best = &kv.first;
      }
    const int64_t len = best ? (int64_t)best->size() : 0;
    if (len >= 1 && len <= 16) {
      int32_t c[16] = {};
      for (int64_t k = 0; k < len; ++k) c[k] = (int32_t)(*best)[k];
      const int64_t rc = 0;
      PatOff po{};
      po.len = (int32_t)len;
      for (int k = 0; k < 16; ++k) po.off[k] = k < len ? (int32_t)(c[k] - rc) : 0;
      if (ls.pat_flag.n < (size_t)ls.n_rows) ls.pat_flag.alloc(ls.n_rows);
      if (!ls.pat_cnt.p) ls.pat_cnt.alloc(1);
      AFEM_HIP(hipMemsetAsync(ls.pat_cnt.p, 0, ls.pat_cnt.bytes(), ctx.stream));
      const unsigned pf_blocks = (unsigned)std::min<int64_t>(8 * 256 * 4, grid_for(16 * ls.n_rows, 256));
      hipLaunchKernelGGL(k_pat_flags, dim3(pf_blocks), dim3(256), 0, ctx.stream, ls.n_rows, ls.csr_rows, ls.csr_cols,
                         po, ls.pat_flag.p, ls.pat_cnt.p);
      AFEM_LAUNCHED();
      unsigned long long hc = 0;
      AFEM_HIP(hipMemcpyAsync(&hc, ls.pat_cnt.p, sizeof(hc), hipMemcpyDeviceToHost, ctx.stream));
      ctx.sync();
      if (hc * 2 >= (unsigned long long)ls.n_rows) {
        pl.rpb = -3;
        pl.po = po;
        pl.pat_flag = ls.pat_flag.p;
        // row blocks of 64 (the default: one wave per block, 7.7 KB of LDS, its barriers
        // wave-local): C2 0.503 vs 0.536 ms per CG iteration with 256, C4 5.64 vs 6.02
        // (r05am, one process); AFEM_SPMV_BS=128 / 256 the larger blocks
        const char* be = variant("AFEM_SPMV_BS");
        const int bsz = be ? atoi(be) : 64;
        if (bsz == 128 || bsz == 64) {
          DevBuf<unsigned long long> mx;
          mx.alloc(1);
          AFEM_HIP(hipMemsetAsync(mx.p, 0, mx.bytes(), ctx.stream));
          const int64_t nb128 = (ls.n_rows + bsz - 1) / bsz;
          hipLaunchKernelGGL(k_block_seg, dim3(grid_for(nb128, 256)), dim3(256), 0, ctx.stream, ls.n_rows, bsz,
                             ls.csr_rows, mx.p);
          AFEM_LAUNCHED();
          unsigned long long hm = 0;
          AFEM_HIP(hipMemcpyAsync(&hm, mx.p, sizeof(hm), hipMemcpyDeviceToHost, ctx.stream));
          ctx.sync();
          if (hm + 3 <= (unsigned long long)(4 * bsz * kSpmvU)) {
            pl.bs = bsz;
            pl.max_seg = (int64_t)hm;
            pl.nblocks = nb128;
          }
        }
        return pl;
      }
    }
  }
  if ((ls.blk_k == 2 || ls.blk_k == 3) && ls.blk_rows && ls.blk_n * ls.blk_k == ls.n_rows && ls.blk_n > 0 && !e) {
    pl.rpb = -2;
    pl.blk_k = ls.blk_k;
    pl.blk_n = ls.blk_n;
    pl.blk_rows = ls.blk_rows;
    pl.blk_cols = ls.blk_cols;
    pl.nblocks = (ls.blk_n + 16 * kBlkRpg - 1) / (16 * kBlkRpg);
  }
  return pl;
}

void launch_spmv(Ctx& ctx, const SpmvPlan& pl, int64_t n_rows, const int64_t* rows, const int32_t* cols,
                 const double* vals, const double* x, double* y, double* partial, int64_t nnz = 0)
{
  const unsigned nb = (unsigned)pl.nblocks;
  if (pl.rpb == -2) {
#define AFEM_BLK(K_)                                                                                               \
  if (partial)                                                                                                    \
    hipLaunchKernelGGL((k_spmv_blk<K_, true>), dim3(nb), dim3(256), 0, ctx.stream, pl.blk_n, pl.blk_rows,         \
                       pl.blk_cols, vals, x, y, partial);                                                         \
  else                                                                                                            \
    hipLaunchKernelGGL((k_spmv_blk<K_, false>), dim3(nb), dim3(256), 0, ctx.stream, pl.blk_n, pl.blk_rows,        \
                       pl.blk_cols, vals, x, y, partial);
    if (pl.blk_k == 3) {
      AFEM_BLK(3)
    }
    else {
      AFEM_BLK(2)
    }
#undef AFEM_BLK
  }
  else if (pl.rpb == -3) {
    const size_t shm = (size_t)(8 * pl.max_seg + 32);
    if (pl.bs == 128 || pl.bs == 64) {
      // (held to 6 / 8 waves per SIMD by a VGPR cap it spills: 0.648 / 1.296 vs 0.507 ms per CG
      // iteration, r05aq)
      auto* kern = pl.bs == 128 ? (partial ? &k_spmv_pat<true, 128> : &k_spmv_pat<false, 128>)
                                : (partial ? &k_spmv_pat<true, 64> : &k_spmv_pat<false, 64>);
      hipLaunchKernelGGL(kern, dim3(nb), dim3(pl.bs), shm, ctx.stream, n_rows, nnz, rows, cols, vals, pl.pat_flag,
                         pl.po, x, y, partial, pl.max_seg, nullptr);
    }
    else if (partial)
      hipLaunchKernelGGL(k_spmv_pat<true>, dim3(nb), dim3(kThreads), shm, ctx.stream, n_rows, nnz, rows, cols, vals,
                         pl.pat_flag, pl.po, x, y, partial, pl.max_seg);
    else
      hipLaunchKernelGGL(k_spmv_pat<false>, dim3(nb), dim3(kThreads), shm, ctx.stream, n_rows, nnz, rows, cols, vals,
                         pl.pat_flag, pl.po, x, y, partial, pl.max_seg);
  }
  else if (pl.rpb < 0) {
    if (partial)
      hipLaunchKernelGGL(k_spmv_v16<true>, dim3(nb), dim3(256), 0, ctx.stream, n_rows, rows, cols, vals, x, y, partial);
    else
      hipLaunchKernelGGL(k_spmv_v16<false>, dim3(nb), dim3(256), 0, ctx.stream, n_rows, rows, cols, vals, x, y,
                         partial);
  }
  else if (pl.rpb && pl.wide && pl.unroll) {
    if (pl.bs == 64 || pl.bs == 128) {
      auto* kern = pl.bs == 64 ? (partial ? &k_spmv_stream4u<true, 64> : &k_spmv_stream4u<false, 64>)
                               : (partial ? &k_spmv_stream4u<true, 128> : &k_spmv_stream4u<false, 128>);
      hipLaunchKernelGGL(kern, dim3(nb), dim3(pl.bs), (size_t)pl.max_seg * 8, ctx.stream, n_rows, nnz, rows, cols,
                         vals, x, y, partial, nullptr);
    }
    else if (partial)
      hipLaunchKernelGGL(k_spmv_stream4u<true>, dim3(nb), dim3(kThreads), (size_t)pl.max_seg * 8, ctx.stream, n_rows,
                         nnz, rows, cols, vals, x, y, partial);
    else
      hipLaunchKernelGGL(k_spmv_stream4u<false>, dim3(nb), dim3(kThreads), (size_t)pl.max_seg * 8, ctx.stream, n_rows,
                         nnz, rows, cols, vals, x, y, partial);
  }
  else if (pl.rpb && pl.wide) {
    if (partial)
      hipLaunchKernelGGL(k_spmv_stream4<true>, dim3(nb), dim3(kThreads), (size_t)pl.max_seg * 8, ctx.stream, n_rows,
                         nnz, rows, cols, vals, x, y, partial);
    else
      hipLaunchKernelGGL(k_spmv_stream4<false>, dim3(nb), dim3(kThreads), (size_t)pl.max_seg * 8, ctx.stream, n_rows,
                         nnz, rows, cols, vals, x, y, partial);
  }
  else if (pl.rpb) {
    if (partial)
      hipLaunchKernelGGL(k_spmv_stream<true>, dim3(nb), dim3(kThreads), (size_t)pl.max_seg * 8, ctx.stream, n_rows,
                         rows, cols, vals, x, y, partial);
    else
      hipLaunchKernelGGL(k_spmv_stream<false>, dim3(nb), dim3(kThreads), (size_t)pl.max_seg * 8, ctx.stream, n_rows,
                         rows, cols, vals, x, y, partial);
  }
  else {
    if (partial)
      hipLaunchKernelGGL(k_spmv_row<true>, dim3(nb), dim3(kThreads), 0, ctx.stream, n_rows, rows, cols, vals, x, y,
                         partial);
    else
      hipLaunchKernelGGL(k_spmv_row<false>, dim3(nb), dim3(kThreads), 0, ctx.stream, n_rows, rows, cols, vals, x, y,
                         partial);
  }
  AFEM_LAUNCHED();
}

// partial[0, n) -> *out.  Long partial arrays (the SpMV's block partials: 390 k at
// C4, 3.1 MB for one workgroup: 37 us per reduce, 2 per CG iteration) go
// through a first pass of kReduceChunks workgroups into scratch[0,
// kReduceChunks) (each a contiguous chunk, fixed order: deterministic).
constexpr int64_t kReduceChunks = 128;
void reduce_to(Ctx& ctx, const double* partial, int64_t n, double* out, double* scratch = nullptr)
{
  const char* e2 = scratch ? variant("AFEM_REDUCE_2STAGE") : nullptr;  // =0: one workgroup (A/B)
  if (scratch && !(e2 && e2[0] == '0') && n > 64 * 1024) {
    hipLaunchKernelGGL(k_reduce_chunks, dim3((unsigned)kReduceChunks), dim3(1024), 0, ctx.stream, n, partial, scratch);
    AFEM_LAUNCHED();
    partial = scratch;
    n = kReduceChunks;
  }
  hipLaunchKernelGGL(k_reduce, dim3(1), dim3(1024), 0, ctx.stream, n, partial, out);
  AFEM_LAUNCHED();
}

void require_csr(LinearSystem& ls)
{
  AFEM_REQUIRE(ls.has_csr, AFEM_ERR_STATE, "linear system has no matrix (setCSRValues / toLinearSystem / matrixAddValue)");
}

}  // namespace

void ls_set_list(LinearSystem& ls, const int32_t* ids, int64_t n, int mem, int kind, double value, double penalty,
                 const double* dvalues)
{
  Ctx& ctx = *ls.ctx;
  if (n <= 0) return;
  const int32_t* dids = ids;
  DevBuf<int32_t> tmp;
  if (mem == AFEM_MEM_HOST) {
    tmp.alloc(n);
    AFEM_HIP(hipMemcpyAsync(tmp.p, ids, tmp.bytes(), hipMemcpyHostToDevice, ctx.stream));
    dids = tmp.p;
  }
  AFEM_REQUIRE(!dvalues || mem == AFEM_MEM_DEVICE, AFEM_ERR_ARG, "ls_set_list: per-DoF values need device ids");
  hipLaunchKernelGGL(k_set_list, dim3(grid_for(n, kThreads)), dim3(kThreads), 0, ctx.stream, n, dids, kind, value,
                     dvalues, penalty, ls.n_rows, ls.forced_info.p, ls.forced_value.p, ls.elim_info.p, ls.elim_value.p,
                     ls.rhs.p);
  AFEM_LAUNCHED();
  if (tmp.p) ctx.sync();
}

void ls_point_update(LinearSystem& ls, int32_t row, int32_t col, double v, bool set)
{
  Ctx& ctx = *ls.ctx;
  AFEM_REQUIRE(row >= 0 && row < ls.csr_n, AFEM_ERR_ARG, "matrix{Add,Set}Value: row out of range");
  DevBuf<int32_t> found;
  found.alloc(1);
  hipLaunchKernelGGL(k_point_update, dim3(1), dim3(64), 0, ctx.stream, ls.csr_rows, ls.csr_cols, ls.csr_vals, row,
                     col, v, set ? 1 : 0, found.p);
  AFEM_LAUNCHED();
  int32_t h = 0;
  AFEM_HIP(hipMemcpyAsync(&h, found.p, sizeof(h), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  AFEM_REQUIRE(h == 1, AFEM_ERR_NOT_FOUND, "matrix{Add,Set}Value: (row,col) is not in the CSR structure");
}

void ls_build_from_host_coo(LinearSystem& ls)
{
  // Aleph semantics: set values override added ones; eliminated rows are
  // handled by the BC kernels (elimination info set from the host map).
  Ctx& ctx = *ls.ctx;
  std::map<std::pair<int32_t, int32_t>, double> merged = ls.add_map;
  for (auto& kv : ls.set_map) merged[kv.first] = kv.second;
  // rows must contain their diagonal for the Jacobi preconditioner
  for (int64_t r = 0; r < ls.n_rows; ++r) merged.emplace(std::make_pair((int32_t)r, (int32_t)r), 0.0);
  std::vector<int64_t> rows(ls.n_rows + 1, 0);
  std::vector<int32_t> cols;
  std::vector<double> vals;
  cols.reserve(merged.size());
  vals.reserve(merged.size());
  for (auto& kv : merged) {
    int32_t r = kv.first.first;
    AFEM_REQUIRE(r >= 0 && r < ls.n_rows, AFEM_ERR_ARG, "matrixAddValue: row out of range");
    AFEM_REQUIRE(kv.first.second >= 0 && kv.first.second < ls.n_cols, AFEM_ERR_ARG,
                 "matrixAddValue: column out of range");
    rows[r + 1]++;
    cols.push_back(kv.first.second);
    vals.push_back(kv.second);
  }
  for (int64_t r = 0; r < ls.n_rows; ++r) rows[r + 1] += rows[r];
  ls.own_rows.alloc(rows.size());
  ls.own_cols.alloc(cols.size());
  ls.own_vals.alloc(vals.size());
  AFEM_HIP(hipMemcpyAsync(ls.own_rows.p, rows.data(), ls.own_rows.bytes(), hipMemcpyHostToDevice, ctx.stream));
  AFEM_HIP(hipMemcpyAsync(ls.own_cols.p, cols.data(), ls.own_cols.bytes(), hipMemcpyHostToDevice, ctx.stream));
  AFEM_HIP(hipMemcpyAsync(ls.own_vals.p, vals.data(), ls.own_vals.bytes(), hipMemcpyHostToDevice, ctx.stream));
  // host eliminations -> device info arrays
  for (auto& kv : ls.host_elim) {
    int32_t d = kv.first;
    uint8_t info = kv.second.first;
    double v = kv.second.second;
    AFEM_HIP(hipMemcpyAsync(ls.elim_info.p + d, &info, 1, hipMemcpyHostToDevice, ctx.stream));
    AFEM_HIP(hipMemcpyAsync(ls.elim_value.p + d, &v, sizeof(double), hipMemcpyHostToDevice, ctx.stream));
    ctx.sync();
  }
  ctx.sync();
  ls.has_csr = true;
  ls.csr_from_coo = true;
  ls.mv_vals = nullptr;
  ls.csr_n = ls.n_rows;
  ls.csr_nnz = (int64_t)cols.size();
  ls.csr_rows = ls.own_rows.p;
  ls.csr_diag = nullptr;
  ls.csr_cols = ls.own_cols.p;
  ls.csr_vals = ls.own_vals.p;
  ls.blk_k = 0;
  ls.mg_k = 0;
  ls.mg.reset();
  ls.amg.reset();
}

void ls_apply_bcs(LinearSystem& ls)
{
  Ctx& ctx = *ls.ctx;
  require_csr(ls);
  // row+column elimination needs a column pass first (only when present)
  bool has_rc = false;
  for (auto& kv : ls.host_elim)
    if (kv.second.first == kElimRowCol) has_rc = true;
  if (has_rc) {
    hipLaunchKernelGGL(k_elim_columns, dim3(grid_for(ls.n_rows, kThreads)), dim3(kThreads), 0, ctx.stream, ls.n_rows,
                       ls.csr_rows, ls.csr_cols, ls.csr_vals, ls.elim_info.p, ls.elim_value.p, ls.rhs.p);
    AFEM_LAUNCHED();
  }
  hipLaunchKernelGGL(k_apply_bcs, dim3(grid_for((ls.n_rows + 3) / 4, kThreads)), dim3(kThreads), 0, ctx.stream, ls.n_rows,
                     ls.csr_rows, ls.csr_cols, ls.csr_vals, ls.forced_info.p, ls.forced_value.p, ls.elim_info.p,
                     ls.elim_value.p, ls.rhs.p, ls.csr_diag);
  AFEM_LAUNCHED();
}

// y = A x with the plan of the current solve (single rank, no halo): the
// algebraic multigrid's fine-level products run the PCG's own SpMV kernel
void ls_spmv_planned(LinearSystem& ls, const double* x, double* y)
{
  AFEM_REQUIRE(ls.spmv_plan, AFEM_ERR_STATE, "no SpMV plan (outside a solve)");
  const SpmvPlan& pl = *static_cast<const SpmvPlan*>(ls.spmv_plan.get());
  launch_spmv(*ls.ctx, pl, ls.n_rows, ls.csr_rows, ls.csr_cols, ls.csr_vals, x, y, nullptr, ls.csr_nnz);
}

void ls_spmv(LinearSystem& ls, const double* x, double* y)
{
  Ctx& ctx = *ls.ctx;
  require_csr(ls);
  if (ls.halo) halo_exchange(*ls.halo, ctx, const_cast<double*>(x));
  SpmvPlan pl = plan_spmv_ls(ctx, ls);
  launch_spmv(ctx, pl, ls.n_rows, ls.csr_rows, ls.csr_cols, ls.csr_vals, x, y, nullptr, ls.csr_nnz);
}

namespace {
void ls_solve_direct(LinearSystem& ls, afem_solve_stats* st)
{
  Ctx& ctx = *ls.ctx;
  const int64_t n = ls.n_rows;
  AFEM_REQUIRE(n <= 4096, AFEM_ERR_LIMIT, "direct solver: more than 4096 rows (use the PCG)");
  ls.dense.alloc((size_t)n * (n + 1));
  if (ls.partial.n < 2 * 64) ls.partial.alloc(2 * 64);
  DevBuf<int> sing;
  sing.alloc(1);
  AFEM_HIP(hipEventRecord(ctx.ev0, ctx.stream));
  hipLaunchKernelGGL(k_csr_to_dense, dim3(grid_for(n, 256)), dim3(256), 0, ctx.stream, n, ls.csr_rows, ls.csr_cols,
                     ls.csr_vals, ls.rhs.p, ls.dense.p);
  AFEM_LAUNCHED();
  hipLaunchKernelGGL(k_dense_gauss, dim3(1), dim3(kDirectThreads), 0, ctx.stream, (int)n, ls.dense.p, ls.sol.p, sing.p);
  AFEM_LAUNCHED();
  AFEM_HIP(hipEventRecord(ctx.ev1, ctx.stream));
  hipLaunchKernelGGL(k_residual, dim3(64), dim3(256), 0, ctx.stream, n, ls.csr_rows, ls.csr_cols, ls.csr_vals,
                     ls.sol.p, ls.rhs.p, ls.partial.p);
  AFEM_LAUNCHED();
  double h[128];
  int hs = 0;
  AFEM_HIP(hipMemcpyAsync(h, ls.partial.p, sizeof(h), hipMemcpyDeviceToHost, ctx.stream));
  AFEM_HIP(hipMemcpyAsync(&hs, sing.p, sizeof(hs), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  ls.dense.reset();
  AFEM_REQUIRE(!hs, AFEM_ERR_ARG, "direct solver: the matrix is singular");
  double rr = 0.0, bb = 0.0;
  for (int i = 0; i < 64; ++i) {
    rr += h[2 * i];
    bb += h[2 * i + 1];
  }
  float ms = 0.f;
  AFEM_HIP(hipEventElapsedTime(&ms, ctx.ev0, ctx.ev1));
  if (st) {
    st->iterations = 0;
    st->converged = 1;
    st->rel_residual = bb > 0 ? std::sqrt(rr / bb) : 0.0;
    st->residual_norm = std::sqrt(rr);
    st->solve_ms = ms;
    st->spmv_kernel = AFEM_SPMV_OTHER;
  }
}
}  // namespace

void ls_solve(LinearSystem& ls, afem_solve_stats* st)
{
  Ctx& ctx = *ls.ctx;
  ctx.set_device();
  if (!ls.has_csr && (!ls.add_map.empty() || !ls.set_map.empty() || !ls.host_elim.empty()))
    ls_build_from_host_coo(ls);
  require_csr(ls);
  AFEM_REQUIRE(ls.csr_n == ls.n_rows, AFEM_ERR_ARG, "CSR view row count differs from the linear system size");
  ls_apply_bcs(ls);
  const bool multi = ls.halo && ls.halo->comm && (comm_nranks(ls.halo->comm) > 1 || comm_self_loop());
  int method = ls.opts.method;
  if (method == AFEM_SOLVER_AUTO)  // femutils/DoFLinearSystem.cc:127-136: direct below 500 rows
    method = (!multi && ls.n_rows < 500 && ls.opts.fixed_iterations <= 0) ? AFEM_SOLVER_DIRECT : AFEM_SOLVER_PCG;
  if (method == AFEM_SOLVER_DIRECT) {
    AFEM_REQUIRE(!multi, AFEM_ERR_NOT_IMPL, "the direct solver runs on one rank (the reference's Sequential "
                                            "solver refuses parallel runs, femutils/DoFLinearSystem.cc:562-564)");
    ls_solve_direct(ls, st);
    return;
  }

  const int64_t n = ls.n_rows;
  if (ls.r.n != (size_t)n) {
    ls.r.alloc(n);
    ls.z.alloc(n);
    ls.q.alloc(n);
    ls.dinv.alloc(n);
    ls.p.alloc(ls.n_cols);
    AFEM_HIP(hipMemsetAsync(ls.p.p, 0, ls.p.bytes(), ctx.stream));
  }
  SpmvPlan pl = plan_spmv_ls(ctx, ls);
  ls.spmv_plan = std::make_shared<SpmvPlan>(pl);  // the preconditioners' fine-level products (amg.hip)
  const int64_t n_part = 2 * std::max<int64_t>(pl.nblocks, kVecBlocks);
  if (ls.partial.n < (size_t)n_part) ls.partial.alloc(n_part);
  if (ls.cons.n != (size_t)n) ls.cons.alloc(n);
  if (ls.scal.n < 8) ls.scal.alloc(8);
  if (!ls.pinned) AFEM_HIP(hipHostMalloc(reinterpret_cast<void**>(&ls.pinned), 8 * sizeof(double), hipHostMallocDefault));
  const unsigned vb = (unsigned)std::min<int64_t>(kVecBlocks, std::max<int64_t>(1, (n + kThreads - 1) / kThreads));

  AFEM_HIP(hipEventRecord(ctx.ev0, ctx.stream));
  if (pl.rpb == -2 && pl.blk_k == 3)
    hipLaunchKernelGGL(k_inv_diag_blk<3>, dim3(grid_for(16 * pl.blk_n, 256)), dim3(256), 0, ctx.stream, pl.blk_n,
                       pl.blk_rows, pl.blk_cols, ls.csr_vals, ls.dinv.p, ls.cons.p);
  else if (pl.rpb == -2 && pl.blk_k == 2)
    hipLaunchKernelGGL(k_inv_diag_blk<2>, dim3(grid_for(16 * pl.blk_n, 256)), dim3(256), 0, ctx.stream, pl.blk_n,
                       pl.blk_rows, pl.blk_cols, ls.csr_vals, ls.dinv.p, ls.cons.p);
  else
    hipLaunchKernelGGL(k_inv_diag, dim3((unsigned)std::min<int64_t>(8 * 256 * 8, grid_for(16 * n, 256))), dim3(256), 0,
                       ctx.stream, n, ls.csr_rows,
                       ls.csr_cols, ls.csr_vals, ls.dinv.p, ls.cons.p);
  AFEM_LAUNCHED();
  const bool blk3 = ls.opts.precond_block == 3;
  AFEM_REQUIRE(!blk3 || n % 3 == 0, AFEM_ERR_ARG, "block-Jacobi 3: the row count is not a multiple of 3");
  const int64_t nb3 = n / 3;
  const unsigned vb3 = (unsigned)std::min<int64_t>(kVecBlocks, std::max<int64_t>(1, (nb3 + kThreads - 1) / kThreads));
  if (blk3) {
    if (ls.binv.n != (size_t)(9 * nb3)) ls.binv.alloc(9 * nb3 > 0 ? 9 * nb3 : 1);
    hipLaunchKernelGGL(k_inv_block3, dim3(grid_for(nb3, 256)), dim3(256), 0, ctx.stream, nb3, ls.csr_rows,
                       ls.csr_cols, ls.csr_vals, ls.cons.p, ls.dinv.p, ls.binv.p);
    AFEM_LAUNCHED();
  }
  // geometric multigrid (structured box, one rank); other systems: point Jacobi
  // (several ranks: block-Jacobi V-cycles on the slabs' owned blocks, mg_available)
  const bool use_gmg = ls.opts.multigrid != 0 && !blk3 && mg_available(ls);
  // algebraic multigrid where the geometric hierarchy does not exist (any mesh, one rank)
  const bool use_amg = !use_gmg && ls.opts.amg != 0 && !blk3 && amg_available(ls);
  const bool use_mg = use_gmg || use_amg;
  if (use_gmg) mg_setup(ls);
  double amg_setup_ms = 0.0;
  if (use_amg) {
    const auto t0 = std::chrono::steady_clock::now();
    if (amg_setup(ls))
      amg_setup_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  // the K-cycle makes the preconditioner nonlinear (its Krylov weights depend
  // on r): the flexible beta then (AFEM_CG_FLEX=0: Fletcher-Reeves)
  const char* fxe = variant("AFEM_CG_FLEX");
  const bool flex = use_amg && amg_nonlinear(ls) && !(fxe && atoi(fxe) == 0);
  // with afem_solver_opts.profile_comm the applications are timed (event pairs, prof_pc below)
  std::function<void(const double*, double*)> precond_timed;
  auto precond = [&](const double* rr, double* zz) {
    if (precond_timed) {
      precond_timed(rr, zz);
      return;
    }
    if (use_amg)
      amg_apply(ls, rr, zz);
    else
      mg_apply(ls, rr, zz);
  };
  // r = b - A x0, z = M^-1 r, p = z and the r.z partials (all rows, free rows)
  auto cg_init = [&]() {
    if (use_mg) {
      hipLaunchKernelGGL(k_cg_init, dim3(vb), dim3(kThreads), 0, ctx.stream, n, ls.rhs.p, ls.q.p, ls.r.p, ls.z.p,
                         ls.p.p, ls.dinv.p, ls.cons.p, ls.partial.p, ls.partial.p + vb);
      AFEM_LAUNCHED();
      precond(ls.r.p, ls.z.p);
      AFEM_HIP(hipMemcpyAsync(ls.p.p, ls.z.p, n * sizeof(double), hipMemcpyDeviceToDevice, ctx.stream));
      // r.z over all rows for both references (the constraint rows' z is r_i / a_ii: negligible)
      hipLaunchKernelGGL(k_dot, dim3(vb), dim3(kThreads), 0, ctx.stream, n, ls.r.p, ls.z.p, ls.partial.p);
      hipLaunchKernelGGL(k_dot, dim3(vb), dim3(kThreads), 0, ctx.stream, n, ls.r.p, ls.z.p, ls.partial.p + vb);
      AFEM_LAUNCHED();
      return;
    }
    if (blk3)
      hipLaunchKernelGGL(k_cg_init_b3, dim3(vb3), dim3(kThreads), 0, ctx.stream, nb3, ls.rhs.p, ls.q.p, ls.r.p,
                         ls.z.p, ls.p.p, ls.binv.p, ls.cons.p, ls.partial.p, ls.partial.p + vb);
    else
      hipLaunchKernelGGL(k_cg_init, dim3(vb), dim3(kThreads), 0, ctx.stream, n, ls.rhs.p, ls.q.p, ls.r.p, ls.z.p,
                         ls.p.p, ls.dinv.p, ls.cons.p, ls.partial.p, ls.partial.p + vb);
    AFEM_LAUNCHED();
  };
  const bool warm = ls.opts.initial_guess == 1;
  if (warm) {  // keep the caller's guess (the cold pass below overwrites the solution)
    if (ls.x0.n != (size_t)n) ls.x0.alloc(n);
    AFEM_HIP(hipMemcpyAsync(ls.x0.p, ls.sol.p, n * sizeof(double), hipMemcpyDeviceToDevice, ctx.stream));
  }
  hipLaunchKernelGGL(k_cg_x0, dim3(vb), dim3(kThreads), 0, ctx.stream, n, ls.rhs.p, ls.dinv.p, ls.cons.p, ls.sol.p,
                     ls.p.p);
  AFEM_LAUNCHED();
  if (ls.halo) halo_exchange(*ls.halo, ctx, ls.p.p);
  launch_spmv(ctx, pl, n, ls.csr_rows, ls.csr_cols, ls.csr_vals, ls.p.p, ls.q.p, nullptr, ls.csr_nnz);
  cg_init();
  double* scal = ls.scal.p;  // [0],[1]: r.z ping-pong, [2]: p.q, [3]: r0.z0 over free rows, [4]: r.r
  reduce_to(ctx, ls.partial.p, blk3 ? vb3 : vb, scal + 0);
  reduce_to(ctx, ls.partial.p + vb, blk3 ? vb3 : vb, scal + 3);
  Comm* comm = ls.halo ? ls.halo->comm : nullptr;
  if (comm) {
    comm_allreduce(comm, ctx, scal + 0, 1);
    comm_allreduce(comm, ctx, scal + 3, 1);
  }
  AFEM_HIP(hipMemcpyAsync(ls.pinned, scal, 4 * sizeof(double), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  // reference value of the stopping test: r0.z0 over the free rows (all rows
  // if every row is a constraint)
  double rz0 = ls.pinned[3] > 0.0 ? ls.pinned[3] : ls.pinned[0];
  if (warm) {
    // start from the caller's guess; the stopping reference stays the one of
    // the zero (lifted) guess above, so the stopping test asks for the same
    // residual as a cold start
    hipLaunchKernelGGL(k_cg_x0_guess, dim3(vb), dim3(kThreads), 0, ctx.stream, n, ls.rhs.p, ls.dinv.p, ls.cons.p,
                       ls.x0.p, ls.sol.p, ls.p.p);
    AFEM_LAUNCHED();
    if (ls.halo) halo_exchange(*ls.halo, ctx, ls.p.p);
    launch_spmv(ctx, pl, n, ls.csr_rows, ls.csr_cols, ls.csr_vals, ls.p.p, ls.q.p, nullptr, ls.csr_nnz);
    cg_init();
    reduce_to(ctx, ls.partial.p, blk3 ? vb3 : vb, scal + 0);
    if (comm) comm_allreduce(comm, ctx, scal + 0, 1);
    AFEM_HIP(hipMemcpyAsync(ls.pinned, scal, sizeof(double), hipMemcpyDeviceToHost, ctx.stream));
    ctx.sync();
  }

  const afem_solver_opts& o = ls.opts;
  const bool fixed = o.fixed_iterations > 0;
  const int max_it = fixed ? o.fixed_iterations : o.max_iter;
  // a multigrid iteration costs ~5 SpMVs: test every 2 iterations (a host sync is ~20 us)
  const int check = use_mg ? std::min(o.check_every > 0 ? o.check_every : 8, 2) : (o.check_every > 0 ? o.check_every : 8);
  double rel = rz0 > 0 ? std::sqrt(std::fabs(ls.pinned[0] / rz0)) : 0.0;
  int it = 0;
  bool converged = fixed ? false : (ls.pinned[0] == 0.0 || rel <= o.rtol);
  // multi-rank: the row blocks that read no ghost column run while the halo
  // of p is in flight (RCCL on the halo's stream), the rest after it lands
  // (host transport: on a worker thread between halo_begin and halo_end with
  // afem_comm_host_async, else inside halo_begin; same split either way)
  const bool overlap = multi && ((pl.rpb > 0 && pl.wide && pl.unroll) || pl.rpb == -2 || pl.rpb == -3);
  int64_t n_int = 0;
  if (overlap) {
    // scalar rows per launch block: kThreads (CSR-stream), pl.bs (pattern) or K * 32 (node blocks)
    const int rpb = pl.rpb == -2 ? pl.blk_k * 16 * kBlkRpg : pl.bs;
    const uint64_t key = (uint64_t)(uintptr_t)ls.csr_rows ^ ((uint64_t)(uintptr_t)ls.csr_cols << 1) ^
                         ((uint64_t)n << 40) ^ (uint64_t)ls.csr_nnz ^ ((uint64_t)rpb << 52);
    if (ls.blist_key != key) {
      DevBuf<uint8_t> fl;
      fl.alloc(pl.nblocks);
      hipLaunchKernelGGL(k_block_ghost, dim3((unsigned)pl.nblocks), dim3(256), 0, ctx.stream, n, rpb,
                         ls.csr_rows, ls.csr_cols, fl.p);
      AFEM_LAUNCHED();
      std::vector<uint8_t> hf(pl.nblocks);
      AFEM_HIP(hipMemcpyAsync(hf.data(), fl.p, pl.nblocks, hipMemcpyDeviceToHost, ctx.stream));
      ctx.sync();
      std::vector<int32_t> in, bd;
      for (int64_t b = 0; b < pl.nblocks; ++b) (hf[b] ? bd : in).push_back((int32_t)b);
      // launch position i of a list runs on XCD i % 8: deal each list's
      // contiguous eighths to the XCDs (neighbouring blocks share one L2)
      std::vector<int32_t> lst;
      for (auto* v : { &in, &bd }) {
        const int64_t m = (int64_t)v->size();
        std::vector<int32_t> sw(m);
        for (int64_t i = 0; i < m; ++i) {
          const int64_t q = m >> 3, rem = m & 7, x = i & 7, j = i >> 3;
          sw[i] = (*v)[x * q + (x < rem ? x : rem) + j];
        }
        lst.insert(lst.end(), sw.begin(), sw.end());
      }
      ls.blist.alloc(lst.size() ? lst.size() : 1);
      if (!lst.empty())
        AFEM_HIP(hipMemcpyAsync(ls.blist.p, lst.data(), lst.size() * 4, hipMemcpyHostToDevice, ctx.stream));
      ls.blist_nint = (int64_t)in.size();
      ls.blist_key = key;
    }
    n_int = ls.blist_nint;
  }
  // afem_solver_opts.profile_comm: event pairs around each halo wait and
  // all-reduce of the loop on the context stream, summed in batches: a fixed
  // pool of kProfEvents events, drained (one stream sync) when it is full
  const bool prof = ls.opts.profile_comm != 0 && comm != nullptr;
  // ... and every preconditioner application (multigrid / AMG), any rank count
  const bool prof_pc = ls.opts.profile_comm != 0 && use_mg;
  constexpr size_t kProfEvents = 256;
  size_t prof_used = 0;
  double prof_halo_ms = 0.0, prof_ar_ms = 0.0, prof_pc_ms = 0.0;
  std::vector<std::pair<size_t, size_t>> prof_halo, prof_ar, prof_pcv;
  auto prof_drain = [&]() {
    if (prof_used == 0) return;
    ctx.sync();
    auto sum_ms = [&](const std::vector<std::pair<size_t, size_t>>& v) {
      double t = 0.0;
      for (const auto& e : v) {
        float m = 0.f;
        AFEM_HIP(hipEventElapsedTime(&m, ls.prof_ev[e.first], ls.prof_ev[e.second]));
        t += m;
      }
      return t;
    };
    prof_halo_ms += sum_ms(prof_halo);
    prof_ar_ms += sum_ms(prof_ar);
    prof_pc_ms += sum_ms(prof_pcv);
    prof_halo.clear();
    prof_ar.clear();
    prof_pcv.clear();
    prof_used = 0;
  };
  // start = the first event of a pair: the pool is drained before a pair that would not fit
  auto prof_event = [&](bool start = false) -> size_t {
    if (start && prof_used + 2 > kProfEvents) prof_drain();
    if (prof_used == ls.prof_ev.size()) {
      hipEvent_t e;
      AFEM_HIP(hipEventCreate(&e));
      ls.prof_ev.push_back(e);
    }
    AFEM_HIP(hipEventRecord(ls.prof_ev[prof_used], ctx.stream));
    return prof_used++;
  };
  if (prof_pc)
    precond_timed = [&](const double* rr, double* zz) {
      const size_t a = prof_event(true);
      if (use_amg)
        amg_apply(ls, rr, zz);
      else
        mg_apply(ls, rr, zz);
      prof_pcv.emplace_back(a, prof_event());
    };
  int n_halo_loop = 0, n_ar_loop = 0;
  auto loop_allreduce = [&](double* d) {
    if (!comm) return;
    const size_t a = prof ? prof_event(true) : 0;
    comm_allreduce(comm, ctx, d, 1);
    if (prof) prof_ar.emplace_back(a, prof_event());
    ++n_ar_loop;
  };
  // the part of an iteration after the SpMV (with_spmv: the whole iteration,
  // for the captured graph of the single-rank, non-split path)
  // AFEM_CG_VEC2=0: one row per thread and access in the vector kernels (variant)
  const char* v2e = variant("AFEM_CG_VEC2");
  const bool vec2 = !(v2e && atoi(v2e) == 0);
  const bool vec4 = v2e && atoi(v2e) == 2;  // AFEM_CG_VEC2=2: two 16-B accesses per thread and iteration
  auto rest_of_iteration = [&](int par, bool with_spmv) {
    if (with_spmv)
      launch_spmv(ctx, pl, n, ls.csr_rows, ls.csr_cols, ls.csr_vals, ls.p.p, ls.q.p, ls.partial.p, ls.csr_nnz);
    reduce_to(ctx, ls.partial.p, pl.nblocks, scal + 2, ls.partial.p + pl.nblocks);
    loop_allreduce(scal + 2);
    if (use_mg) {
      hipLaunchKernelGGL(k_cg_xr, dim3(vb), dim3(kThreads), 0, ctx.stream, n, scal, par, ls.sol.p, ls.p.p, ls.r.p,
                         ls.q.p);
      AFEM_LAUNCHED();
      precond(ls.r.p, ls.z.p);
      hipLaunchKernelGGL(k_dot, dim3(vb), dim3(kThreads), 0, ctx.stream, n, ls.r.p, ls.z.p, ls.partial.p);
      if (flex) {
        hipLaunchKernelGGL(k_dot, dim3(vb), dim3(kThreads), 0, ctx.stream, n, ls.z.p, ls.q.p, ls.partial.p + vb);
        reduce_to(ctx, ls.partial.p + vb, vb, scal + 5);
        loop_allreduce(scal + 5);
      }
      AFEM_LAUNCHED();
    }
    else if (blk3)
      hipLaunchKernelGGL(k_cg_update_b3, dim3(vb3), dim3(kThreads), 0, ctx.stream, nb3, scal, par, ls.sol.p, ls.p.p,
                         ls.r.p, ls.q.p, ls.z.p, ls.binv.p, ls.partial.p);
    else
      hipLaunchKernelGGL(vec4 ? (k_cg_update_rz<true, true>) : vec2 ? (k_cg_update_rz<true>) : (k_cg_update_rz<false>), dim3(vb), dim3(kThreads), 0, ctx.stream,
                         n, scal, par, ls.r.p, ls.q.p, ls.z.p, ls.dinv.p, ls.partial.p);
    AFEM_LAUNCHED();
    reduce_to(ctx, ls.partial.p, blk3 ? vb3 : vb, scal + (par ^ 1));
    loop_allreduce(scal + (par ^ 1));
    if (flex)
      hipLaunchKernelGGL(k_cg_dir_flex, dim3(vb), dim3(kThreads), 0, ctx.stream, n, (const double*)scal, ls.z.p,
                         ls.p.p);
    else if (use_mg || blk3)
      hipLaunchKernelGGL(k_cg_dir, dim3(vb), dim3(kThreads), 0, ctx.stream, n, scal, par, ls.z.p, ls.p.p);
    else
      hipLaunchKernelGGL(vec4 ? (k_cg_dir_x<true, true>) : vec2 ? (k_cg_dir_x<true>) : (k_cg_dir_x<false>), dim3(vb), dim3(kThreads), 0, ctx.stream, n, scal,
                         par, ls.sol.p, ls.z.p, ls.p.p);
    AFEM_LAUNCHED();
  };
  // graph replay of whole iterations (single rank, no split SpMV, no
  // multigrid: every launch of an iteration is a plain kernel), in batches of
  // the convergence-check period (even: the ping-pong parity of the scalars
  // repeats).  Opt-in (AFEM_CG_GRAPH=1): measured on MI355X at C2 the replayed
  // batches cost MORE device time than the launched kernels (0.68 vs 0.60 ms
  // per iteration, profiles/r03_v3_bench.json vs r03_v3_cg_nograph_bench.json)
  const char* cgg = variant("AFEM_CG_GRAPH");
  const int gbatch = fixed ? 16 : check;
  const bool graph = !multi && !use_mg && !comm && !overlap && (gbatch % 2) == 0 && gbatch >= 2 &&
                     (cgg && atoi(cgg) == 1);
  hipGraphExec_t gexec = nullptr;
  struct GraphGuard {
    hipGraphExec_t& g;
    ~GraphGuard()
    {
      if (g) (void)hipGraphExecDestroy(g);
    }
  } graph_guard{ gexec };
  while (!converged && it < max_it) {
    const int par = it & 1;
    if (overlap) {
      const int64_t n_bd = pl.nblocks - n_int;
      auto part = [&](int64_t nbk, int64_t off) {
        if (nbk <= 0) return;
        if (pl.rpb == -3) {
          auto* kern = pl.bs == 64 ? &k_spmv_pat<true, 64> : pl.bs == 128 ? &k_spmv_pat<true, 128> : &k_spmv_pat<true>;
          hipLaunchKernelGGL(kern, dim3((unsigned)nbk), dim3(pl.bs), (size_t)(8 * pl.max_seg + 32), ctx.stream, n,
                             ls.csr_nnz, ls.csr_rows, ls.csr_cols, ls.csr_vals, pl.pat_flag, pl.po, ls.p.p, ls.q.p,
                             ls.partial.p + off, pl.max_seg, ls.blist.p + off);
        }
        else if (pl.rpb != -2)
        {
          auto* kern = pl.bs == 64    ? &k_spmv_stream4u<true, 64>
                       : pl.bs == 128 ? &k_spmv_stream4u<true, 128>
                                      : &k_spmv_stream4u<true>;
          hipLaunchKernelGGL(kern, dim3((unsigned)nbk), dim3(pl.bs), (size_t)pl.max_seg * 8, ctx.stream, n,
                             ls.csr_nnz, ls.csr_rows, ls.csr_cols, ls.csr_vals, ls.p.p, ls.q.p, ls.partial.p + off,
                             ls.blist.p + off);
        }
        else if (pl.blk_k == 3)
          hipLaunchKernelGGL((k_spmv_blk<3, true>), dim3((unsigned)nbk), dim3(256), 0, ctx.stream, pl.blk_n,
                             pl.blk_rows, pl.blk_cols, ls.csr_vals, ls.p.p, ls.q.p, ls.partial.p + off,
                             ls.blist.p + off);
        else
          hipLaunchKernelGGL((k_spmv_blk<2, true>), dim3((unsigned)nbk), dim3(256), 0, ctx.stream, pl.blk_n,
                             pl.blk_rows, pl.blk_cols, ls.csr_vals, ls.p.p, ls.q.p, ls.partial.p + off,
                             ls.blist.p + off);
        AFEM_LAUNCHED();
      };
      halo_begin(*ls.halo, ctx, ls.p.p);
      part(n_int, 0);
      const size_t ha = prof ? prof_event(true) : 0;
      halo_end(*ls.halo, ctx, ls.p.p);
      if (prof) prof_halo.emplace_back(ha, prof_event());
      ++n_halo_loop;
      part(n_bd, n_int);
    }
    else if (graph && (it & 1) == 0 && it + gbatch <= max_it) {
      // single rank: `gbatch` whole iterations replayed as one captured graph
      if (!gexec) {
        hipGraph_t g = nullptr;
        AFEM_HIP(hipStreamBeginCapture(ctx.stream, hipStreamCaptureModeThreadLocal));
        for (int b = 0; b < gbatch; ++b) rest_of_iteration(b & 1, true);
        AFEM_HIP(hipStreamEndCapture(ctx.stream, &g));
        const hipError_t e = hipGraphInstantiate(&gexec, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        AFEM_HIP(e);
      }
      AFEM_HIP(hipGraphLaunch(gexec, ctx.stream));
      it += gbatch - 1;  // the last one is counted below
      ++it;
      goto checked;
    }
    else {
      if (ls.halo) {
        const size_t ha = prof ? prof_event(true) : 0;
        halo_exchange(*ls.halo, ctx, ls.p.p);
        if (prof) prof_halo.emplace_back(ha, prof_event());
        ++n_halo_loop;
      }
      launch_spmv(ctx, pl, n, ls.csr_rows, ls.csr_cols, ls.csr_vals, ls.p.p, ls.q.p, ls.partial.p, ls.csr_nnz);
    }
    rest_of_iteration(par, false);
    ++it;
  checked:
    if (!fixed && (it % check == 0 || it == max_it)) {
      AFEM_HIP(hipMemcpyAsync(ls.pinned, scal, 4 * sizeof(double), hipMemcpyDeviceToHost, ctx.stream));
      ctx.sync();
      const double rz = ls.pinned[it & 1];
      rel = std::sqrt(std::fabs(rz / rz0));
      if (rel <= o.rtol) converged = true;
      if (!converged && o.atol > 0) {
        hipLaunchKernelGGL(k_dot, dim3(vb), dim3(kThreads), 0, ctx.stream, n, ls.r.p, ls.r.p, ls.partial.p);
        AFEM_LAUNCHED();
        reduce_to(ctx, ls.partial.p, vb, scal + 4);
        if (comm) comm_allreduce(comm, ctx, scal + 4, 1);
        AFEM_HIP(hipMemcpyAsync(ls.pinned + 4, scal + 4, sizeof(double), hipMemcpyDeviceToHost, ctx.stream));
        ctx.sync();
        if (std::sqrt(ls.pinned[4]) <= o.atol) converged = true;
      }
    }
  }
  AFEM_HIP(hipEventRecord(ctx.ev1, ctx.stream));
  // final residual norm (recurrence residual) and relative preconditioned residual
  hipLaunchKernelGGL(k_dot, dim3(vb), dim3(kThreads), 0, ctx.stream, n, ls.r.p, ls.r.p, ls.partial.p);
  AFEM_LAUNCHED();
  reduce_to(ctx, ls.partial.p, vb, scal + 4);
  if (comm) comm_allreduce(comm, ctx, scal + 4, 1);
  AFEM_HIP(hipMemcpyAsync(ls.pinned, scal, 5 * sizeof(double), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  float ms = 0.f;
  AFEM_HIP(hipEventElapsedTime(&ms, ctx.ev0, ctx.ev1));
  rel = rz0 > 0 ? std::sqrt(std::fabs(ls.pinned[it & 1] / rz0)) : 0.0;
  if (ls.halo) halo_exchange(*ls.halo, ctx, ls.sol.p);  // m_u.synchronize()
  if (st) {
    if (prof || prof_pc) prof_drain();
    st->precond_ms = prof_pc ? prof_pc_ms : 0.0;
    st->halo_wait_ms = prof ? prof_halo_ms : 0.0;
    st->allreduce_ms = prof ? prof_ar_ms : 0.0;
    st->halo_bytes = ls.halo ? 8 * ls.halo->n_send : 0;
    st->n_halo = n_halo_loop;
    st->n_allreduce = n_ar_loop;
    st->amg_setup_ms = amg_setup_ms;
    if (use_amg)
      amg_stats(ls, &st->amg_levels, &st->amg_coarse_rows, &st->amg_complexity);
    else {
      st->amg_levels = 0;
      st->amg_coarse_rows = 0;
      st->amg_complexity = 0.0;
    }
    st->iterations = it;
    st->converged = fixed ? (rel <= o.rtol) : converged;
    st->rel_residual = rel;
    st->residual_norm = std::sqrt(std::fabs(ls.pinned[4]));
    st->solve_ms = ms;
    st->spmv_kernel = pl.rpb == -3 ? AFEM_SPMV_PATTERN
                      : pl.rpb == -2 ? AFEM_SPMV_BLOCK
                      : pl.rpb == -1 ? AFEM_SPMV_VECTOR
                      : (pl.rpb > 0 && pl.wide && pl.unroll) ? AFEM_SPMV_STREAM
                                                             : AFEM_SPMV_OTHER;
  }
}

}  // namespace afem
