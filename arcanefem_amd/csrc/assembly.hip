// P1 global-matrix assembly (the hot path; replaces the cell-wise atomic
// scatter of BSRFormat::assembleBilinearOrderedPerBlock/PerRow,
// femutils/BSRFormat.h:786-898, and the RHS source term of
// femutils/ArcaneFemFunctionsGpu.h:401-429).
//
// Design: a workgroup owns a contiguous block of rows,
// i.e. a contiguous segment of the CSR value array.  Each lane owns one row
// and walks the row's incident cells through the row-local incidence table
// (sliced ELL, one coalesced 256-B wave load per step).  An incidence gives
// the row-slots of the cell's other nodes, so the lane recovers their node
// ids from the row's columns (staged in LDS), gathers their coordinates
// (L1/L2/Infinity-Cache resident: each node is a neighbour of ~15 rows),
// recomputes the element row K_e[row node, :] and accumulates it into the
// row's slice of an LDS accumulator.  The diagonal and the RHS are
// accumulated in registers.  The block then streams its finished segment to
// HBM with coalesced stores.  Consequences:
//   * every value is written exactly once, no zero-fill pass, no float
//     atomics (global f64 atomics run at ~1.3 TB/s at best and ~0.08 TB/s
//     when 64 lanes hit 64 rows — the reference's access pattern);
//   * the summation order of every entry is fixed by the structure, so the
//     assembled matrix is bitwise reproducible run to run;
//   * HBM traffic ~= the algorithmic minimum: incidence table (4 B per
//     (cell,node), the same bytes as the connectivity), row offsets, columns,
//     values, RHS, coordinates once.
#include "afem_internal.hpp"

#include <cstdlib>

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
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return V3{ a.x - b.x, a.y - b.y, a.z - b.z }; }
__device__ __forceinline__ V3 cross(V3 a, V3 b)
{
  return V3{ a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x };
}
__device__ __forceinline__ double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

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

// ---------------------------------------------------------------- scalar P1
__host__ __device__ constexpr int64_t lds_acc_bytes(int64_t seg_cap) { return ((8 * (seg_cap + 2)) + 15) & ~int64_t(15); }
__host__ __device__ constexpr int64_t lds_scalar_bytes(int64_t seg_cap)
{
  return (lds_acc_bytes(seg_cap) + 4 * (seg_cap + 8) + 15) & ~int64_t(15);
}
// Incidence entry k of the row in lane `lane` of slice `sl` lives at
// inc[slice_ptr[sl] + (k/4)*256 + lane*4 + k%4]: one 16-B load per lane per 4
// incidences, coalesced over the wave (1 KiB per load instruction).
// Accumulation into the row's LDS slice uses ds_add_f64: a row is owned by a
// single lane and a wave's LDS operations execute in program order, so the
// summation order of every entry is fixed (bitwise reproducible) while the
// read-modify-write latency stays off the lane's dependency chain.
// ABL != 0 only in diagnostic runs (AFEM_ASSEMBLY_ABLATION, results wrong):
// 1 = no element arithmetic, 2 = no coordinate gathers, 3 = no LDS adds.
template <int NV, bool USE_LDS, int ABL = 0>
__global__ __launch_bounds__(256) void k_assemble_p1(int64_t n_rows, int64_t seg_cap,
                                                     const int64_t* __restrict__ row_ptr,
                                                     const int32_t* __restrict__ cols,
                                                     const uint32_t* __restrict__ inc,
                                                     const int64_t* __restrict__ slice_ptr,
                                                     const int32_t* __restrict__ slice_k,
                                                     const double* __restrict__ coords, double s_coef,
                                                     double f_meas, double* __restrict__ vals,
                                                     double* __restrict__ rhs)
{
  // Wave-local: each wave owns one slice of 64 consecutive rows and its own
  // LDS region (accumulators + the slice's columns).  No workgroup barrier:
  // a wave's LDS operations execute in order, so its staging, accumulation
  // and write-back need no synchronisation with the other waves, and the
  // waves of a CU drift through the stage/compute/write phases independently.
  extern __shared__ __align__(16) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  unsigned char* wmem = smem + (size_t)wid * (size_t)lds_scalar_bytes(seg_cap);
  double* acc = reinterpret_cast<double*>(wmem);                                // [seg_cap + 2]
  int32_t* scol = reinterpret_cast<int32_t*>(wmem + lds_acc_bytes(seg_cap));  // [seg_cap + 8]

  const int64_t n_slices = (n_rows + 63) >> 6;
  const int64_t blk = xcd_swizzle(blockIdx.x, gridDim.x);
  const int64_t sl = blk * (int64_t)(blockDim.x >> 6) + wid;
  if (sl >= n_slices) return;  // whole wave: no barrier follows
  const int64_t r0 = sl << 6;
  const int64_t r1 = (r0 + 64 < n_rows) ? r0 + 64 : n_rows;
  const int64_t r = r0 + lane;
  const bool active = r < r1;

  // Per-lane prologue loads first, so their latency overlaps the staging.
  const int64_t seg0 = row_ptr[r0];
  const int64_t seg1 = row_ptr[r1];
  const int64_t rb = active ? row_ptr[r] : seg0;
  const int64_t re = active ? row_ptr[r + 1] : seg0;
  const V3 xi = ld3(coords, active ? r : r0);
  const uint4* ip = reinterpret_cast<const uint4*>(inc + slice_ptr[sl]) + lane;
  const int ngroups = active ? (slice_k[sl] >> 2) : 0;
  uint4 e4 = ngroups > 0 ? ip[0] : make_uint4(kPad, kPad, kPad, kPad);

  // The slice's columns staged in LDS with 16-B loads from the 16-B aligned
  // start (cols carries 4 ints of tail padding), all of a lane's loads issued
  // before its LDS writes; accumulators zeroed with 16-B stores.
  const int64_t q0 = seg0 >> 2;  // first uint4 of the segment
  if (USE_LDS) {
    const int64_t nq = ((seg1 + 3) >> 2) - q0;
    const uint4* src = reinterpret_cast<const uint4*>(cols) + q0;
    uint4* dst = reinterpret_cast<uint4*>(scol);
    for (int64_t q = lane; q < nq; q += 256) {
      const bool b1 = q + 64 < nq, b2 = q + 128 < nq, b3 = q + 192 < nq;
      const uint4 v0 = src[q];
      const uint4 v1 = b1 ? src[q + 64] : make_uint4(0, 0, 0, 0);
      const uint4 v2 = b2 ? src[q + 128] : make_uint4(0, 0, 0, 0);
      const uint4 v3 = b3 ? src[q + 192] : make_uint4(0, 0, 0, 0);
      dst[q] = v0;
      if (b1) dst[q + 64] = v1;
      if (b2) dst[q + 128] = v2;
      if (b3) dst[q + 192] = v3;
    }
    const int64_t n2 = (seg1 - seg0 + 1) >> 1;
    double2* a2 = reinterpret_cast<double2*>(acc);
    for (int64_t t = lane; t < n2; t += 64) a2[t] = make_double2(0.0, 0.0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  if (active) {
    double* arow = USE_LDS ? acc + (rb - seg0) : vals + rb;
    const int32_t* crow = USE_LDS ? scol + (rb - 4 * q0) : cols + rb;
    if (!USE_LDS) {
      for (int64_t t = 0; t < re - rb; ++t) arow[t] = 0.0;
    }
    double dacc = 0.0, macc = 0.0;
    uint32_t dslot = 0xFFu;
    // Branch-free groups of 4 incidences (padding entries become a zero
    // contribution to slot 0), so every LDS read and coordinate gather of
    // the group is issued before the first element row is computed; the
    // next group's incidence word is prefetched one group ahead.
    for (int g = 0; g < ngroups; ++g) {
      const uint4 cur = e4;
      if (cur.x == kPad) break;
      if (g + 1 < ngroups) e4 = ip[(int64_t)(g + 1) * 64];
      const uint32_t ev[4] = { cur.x, cur.y, cur.z, cur.w };
      V3 xa[4], xb[4], xc[4];
      uint32_t sa[4], sb[4], sc[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t e = ev[j] == kPad ? 0u : ev[j];
        sa[j] = e & 0xFFu;
        sb[j] = (e >> 8) & 0xFFu;
        sc[j] = (NV == 4) ? (e >> 16) & 0xFFu : 0u;
        if (ABL == 2) {
          const double da = 1e-3 * (double)crow[sa[j]], db = 2e-3 * (double)crow[sb[j]],
                       dc = 3e-3 * (double)crow[sc[j]];
          xa[j] = V3{ xi.x + da, xi.y, xi.z };
          xb[j] = V3{ xi.x, xi.y + db, xi.z };
          xc[j] = V3{ xi.x, xi.y, xi.z + dc };
        }
        else {
          xa[j] = ld3(coords, crow[sa[j]]);
          xb[j] = ld3(coords, crow[sb[j]]);
          if (NV == 4) xc[j] = ld3(coords, crow[sc[j]]);
        }
      }
      dslot = (cur.x >> 24);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool valid = ev[j] != kPad;
        double k0, k1, k2, k3 = 0.0, meas;
        if (ABL == 1) {
          k0 = xa[j].x;
          k1 = xa[j].y + xb[j].x;
          k2 = xb[j].y + xc[j].x;
          k3 = xc[j].y + xc[j].z;
          meas = xa[j].z + xb[j].z;
        }
        else if (NV == 4)
          meas = tet_row(xi, xa[j], xb[j], xc[j], s_coef, k0, k1, k2, k3);
        else
          meas = tri_row(xi, xa[j], xb[j], s_coef, k0, k1, k2);
        if (!valid) k0 = k1 = k2 = k3 = meas = 0.0;
        dacc += k0;
        macc += meas;
        if (ABL == 3) {
          dacc += k1 + k2 + k3;
        }
        else if (USE_LDS) {
          atomicAdd(arow + sa[j], k1);
          atomicAdd(arow + sb[j], k2);
          if (NV == 4) atomicAdd(arow + sc[j], k3);
        }
        else {
          arow[sa[j]] += k1;
          arow[sb[j]] += k2;
          if (NV == 4) arow[sc[j]] += k3;
        }
      }
    }
    if (dslot != 0xFFu) arow[dslot] = dacc;
    if (rhs) rhs[r] = f_meas * macc;
  }
  if (USE_LDS) {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (int64_t t = lane; t < seg1 - seg0; t += 64) vals[seg0 + t] = acc[t];
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

template <bool USE_LDS>
__global__ __launch_bounds__(256) void k_assemble_elast_tri(int64_t n_rows, int64_t seg_cap, bool per_block,
                                                            const int64_t* __restrict__ row_ptr,
                                                            const int32_t* __restrict__ cols,
                                                            const uint32_t* __restrict__ inc,
                                                            const int64_t* __restrict__ slice_ptr,
                                                            const int32_t* __restrict__ slice_k,
                                                            const double* __restrict__ coords, double lambda,
                                                            double mu2, double* __restrict__ vals)
{
  extern __shared__ __align__(16) unsigned char smem[];
  double* acc = reinterpret_cast<double*>(smem);
  int32_t* scol = reinterpret_cast<int32_t*>(smem + 8 * 4 * seg_cap);
  const int rpb = blockDim.x;
  const int64_t blk = xcd_swizzle(blockIdx.x, gridDim.x);
  const int64_t r0 = blk * rpb;
  const int64_t r1 = (r0 + rpb < n_rows) ? r0 + rpb : n_rows;
  const int64_t seg0 = row_ptr[r0];
  const int64_t r = r0 + threadIdx.x;
  double* out = USE_LDS ? acc : vals;
  const int64_t base0 = USE_LDS ? seg0 * 4 : 0;
  if (USE_LDS) {
    const int64_t seglen = row_ptr[r1] - seg0;
    for (int64_t t = threadIdx.x; t < seglen; t += rpb) scol[t] = cols[seg0 + t];
    for (int64_t t = threadIdx.x; t < 4 * seglen; t += rpb) acc[t] = 0.0;
    __syncthreads();
  }
  if (r < r1) {
    const int64_t rb = row_ptr[r];
    const int64_t nnz_row = row_ptr[r + 1] - rb;
    const int64_t rb4 = rb * 4 - base0;
    if (!USE_LDS)
      for (int64_t t = 0; t < 4 * nnz_row; ++t) vals[rb * 4 + t] = 0.0;
    const V3 x0 = ld3(coords, r);
    const int64_t sl = r >> 6;
    const uint32_t* ip = inc + slice_ptr[sl] + (r & 63) * 4;
    const int kmax = slice_k[sl];
    double d00 = 0, d01 = 0, d10 = 0, d11 = 0;
    uint32_t dslot = 0xFFu;
    for (int k = 0; k < kmax; ++k) {
      const uint32_t e = ip[(int64_t)(k >> 2) * 256 + (k & 3)];
      if (e == kPad) break;
      const int s[2] = { (int)(e & 0xFFu), (int)((e >> 8) & 0xFFu) };
      dslot = e >> 24;
      const int64_t cb = USE_LDS ? (rb - seg0) : rb;
      const int32_t* cc = USE_LDS ? scol : cols;
      const V3 x1 = ld3(coords, cc[cb + s[0]]), x2 = ld3(coords, cc[cb + s[1]]);
      // 2A * grad N: dPhi0 = (y1-y2, x2-x1), dPhi1 = (y2-y0, x0-x2), dPhi2 = (y0-y1, x1-x0)
      const double p0x = x1.y - x2.y, p0y = x2.x - x1.x;
      const double px[3] = { p0x, x2.y - x0.y, x0.y - x1.y };
      const double py[3] = { p0y, x0.x - x2.x, x1.x - x0.x };
      V3 a = sub(x1, x0), b = sub(x2, x0);
      V3 cr = cross(a, b);
      const double area = sqrt(dot(cr, cr)) / 2.0;
      const double sc = 1.0 / (4.0 * area);
      // row dof i of node 0, column dof j of node b:
      //  lam(i,j)  = (bx_i + by_i)(bx_j + by_j) over the interleaved B rows
      //  shr(i,j)  = bx_i bx_j + by_i by_j + 0.5 bs_i bs_j
      // with for dof (node a, comp 0): bx = px[a], by = 0, bs = py[a]
      //      for dof (node a, comp 1): bx = 0, by = py[a], bs = px[a]
      for (int nb = 0; nb < 3; ++nb) {
        double K00, K01, K10, K11;
        {
          // i=0 (u1 of node 0), j=0 (u1 of node nb)
          double lam = px[0] * px[nb];
          double shr = px[0] * px[nb] + 0.5 * py[0] * py[nb];
          K00 = (lambda * lam) * sc + (mu2 * shr) * sc;
          // i=0, j=1 (u2 of node nb)
          lam = px[0] * py[nb];
          shr = 0.5 * py[0] * px[nb];
          K01 = (lambda * lam) * sc + (mu2 * shr) * sc;
          // i=1, j=0
          lam = py[0] * px[nb];
          shr = 0.5 * px[0] * py[nb];
          K10 = (lambda * lam) * sc + (mu2 * shr) * sc;
          // i=1, j=1
          lam = py[0] * py[nb];
          shr = py[0] * py[nb] + 0.5 * px[0] * px[nb];
          K11 = (lambda * lam) * sc + (mu2 * shr) * sc;
        }
        if (nb == 0) {
          d00 += K00;
          d01 += K01;
          d10 += K10;
          d11 += K11;
        }
        else {
          const int sl2 = s[nb - 1];
          out[bidx2(per_block, rb4, nnz_row, sl2, 0, 0)] += K00;
          out[bidx2(per_block, rb4, nnz_row, sl2, 0, 1)] += K01;
          out[bidx2(per_block, rb4, nnz_row, sl2, 1, 0)] += K10;
          out[bidx2(per_block, rb4, nnz_row, sl2, 1, 1)] += K11;
        }
      }
    }
    if (dslot != 0xFFu) {
      out[bidx2(per_block, rb4, nnz_row, (int)dslot, 0, 0)] = d00;
      out[bidx2(per_block, rb4, nnz_row, (int)dslot, 0, 1)] = d01;
      out[bidx2(per_block, rb4, nnz_row, (int)dslot, 1, 0)] = d10;
      out[bidx2(per_block, rb4, nnz_row, (int)dslot, 1, 1)] = d11;
    }
  }
  if (USE_LDS) {
    __syncthreads();
    const int64_t seglen = row_ptr[r1] - seg0;
    for (int64_t t = threadIdx.x; t < 4 * seglen; t += rpb) vals[seg0 * 4 + t] = acc[t];
  }
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

void assemble_scalar(Bsr& b, double coef, double f, double* rhs)
{
  Structure& s = b.s;
  Ctx& ctx = *b.mesh->ctx;
  const int nv = b.mesh->nv;
  AFEM_REQUIRE(b.nb_dof == 1, AFEM_ERR_ARG, "assembleBilinear(P1 Laplacian) needs NB_DOF = 1");
  // wave-local kernel: 4 waves per workgroup, one LDS region per wave
  const int64_t wave_lds = lds_scalar_bytes(s.max_wave_seg);
  const bool lds = 4 * wave_lds <= 64 * 1024;
  const int rpb = 256;
  const unsigned nblk = lds ? (unsigned)((s.n_slices + 3) / 4) : (unsigned)((s.n_rows + rpb - 1) / rpb);
  const size_t shm = lds ? (size_t)(4 * wave_lds) : 0;
  // K = coef * c0.cb / (6|det|) (tets) or / (2|A2|) (triangles);
  // RHS = f * |K| / nv = f*|det|/24 (tets) or f*|A2|/6 (triangles)
  const double s_coef = (nv == 4) ? coef / 6.0 : coef / 2.0;
  const double f_meas = (nv == 4) ? f / 24.0 : f / 6.0;
  static const int abl = [] {
    const char* e = getenv("AFEM_ASSEMBLY_ABLATION");
    return e ? atoi(e) : 0;
  }();
#define AFEM_ASM_ARGS s.n_rows, s.max_wave_seg, s.row_ptr.p, s.cols.p, s.inc.p, s.inc_slice_ptr.p, s.inc_slice_k.p, \
                      b.mesh->coords.p, s_coef, f_meas, b.values.p, rhs
  if (nv == 4 && lds) {
    switch (abl) {
      case 1: hipLaunchKernelGGL((k_assemble_p1<4, true, 1>), dim3(nblk), dim3(rpb), shm, ctx.stream, AFEM_ASM_ARGS); break;
      case 2: hipLaunchKernelGGL((k_assemble_p1<4, true, 2>), dim3(nblk), dim3(rpb), shm, ctx.stream, AFEM_ASM_ARGS); break;
      case 3: hipLaunchKernelGGL((k_assemble_p1<4, true, 3>), dim3(nblk), dim3(rpb), shm, ctx.stream, AFEM_ASM_ARGS); break;
      default: hipLaunchKernelGGL((k_assemble_p1<4, true>), dim3(nblk), dim3(rpb), shm, ctx.stream, AFEM_ASM_ARGS);
    }
  }
  else if (nv == 4)
    hipLaunchKernelGGL((k_assemble_p1<4, false>), dim3(nblk), dim3(rpb), 0, ctx.stream, AFEM_ASM_ARGS);
  else if (lds)
    hipLaunchKernelGGL((k_assemble_p1<3, true>), dim3(nblk), dim3(rpb), shm, ctx.stream, AFEM_ASM_ARGS);
  else
    hipLaunchKernelGGL((k_assemble_p1<3, false>), dim3(nblk), dim3(rpb), 0, ctx.stream, AFEM_ASM_ARGS);
#undef AFEM_ASM_ARGS
  AFEM_LAUNCHED();
}

void assemble_elasticity_tri(Bsr& b, double lambda, double mu2)
{
  Structure& s = b.s;
  Ctx& ctx = *b.mesh->ctx;
  AFEM_REQUIRE(b.nb_dof == 2 && b.mesh->nv == 3, AFEM_ERR_NOT_IMPL,
               "P1 elasticity assembly is implemented for NB_DOF = 2 on triangles (the reference's elasticity module)");
  const bool lds = s.rows_per_block > 0 && s.max_seg * 36 <= 64 * 1024;
  const int rpb = lds ? s.rows_per_block : 256;
  const unsigned nblk = (unsigned)((s.n_rows + rpb - 1) / rpb);
  const size_t shm = lds ? (size_t)s.max_seg * 36 : 0;
  if (lds)
    hipLaunchKernelGGL(k_assemble_elast_tri<true>, dim3(nblk), dim3(rpb), shm, ctx.stream, s.n_rows, s.max_seg,
                       b.order_per_block, s.row_ptr.p, s.cols.p, s.inc.p, s.inc_slice_ptr.p, s.inc_slice_k.p,
                       b.mesh->coords.p, lambda, mu2, b.values.p);
  else
    hipLaunchKernelGGL(k_assemble_elast_tri<false>, dim3(nblk), dim3(rpb), 0, ctx.stream, s.n_rows, s.max_seg,
                       b.order_per_block, s.row_ptr.p, s.cols.p, s.inc.p, s.inc_slice_ptr.p, s.inc_slice_k.p,
                       b.mesh->coords.p, lambda, mu2, b.values.p);
  AFEM_LAUNCHED();
}

}  // namespace afem
