// Geometric multigrid preconditioner for the PCG (afem_solver_opts.multigrid)
// on systems assembled on a structured Kuhn box on one rank (Mesh.structured:
// node (x, y, z) = x + (nx+1)(y + (ny+1) z), every cube split into the six
// tetrahedra around its main diagonal).
//
// The reference's GPU solve is Hypre PCG + BoomerAMG (femutils/
// HypreDoFLinearSystem.cc:387-762); this is the structured-grid counterpart,
// built from the assembled matrix alone (no physics on the coarse levels):
//  * hierarchy: the box with every other node, while the cell counts stay
//    even; the Kuhn triangulation of the half grid is nested in the fine one,
//    so the coarse hat function of node I is the fine-grid function with value
//    1 at node 2I and 1/2 at the 14 fine nodes 2I +- e (e in {0,1}^3 \ 0, the
//    midpoints of the coarse Kuhn edges at I) -- P is that interpolation in
//    index space (exact P1 interpolation without jitter), R = P^T;
//  * coarse operators A_c = P^T A P (Galerkin), formed by a deterministic
//    per-coarse-row kernel on the coarse Kuhn stencil (15 node blocks per row,
//    the exact sparsity of P^T A P for nested Kuhn grids); penalty rows carry
//    over by themselves;
//  * smoothing: damped Jacobi, omega = 4 / (3 lambda_max(D^-1 A)) from a power
//    iteration per level, one sweep before and one after (symmetric V-cycle);
//    block-3 systems run the cycle's products (sweeps, residuals) on fp32 copies
//    of every level's values in a 16-B-per-block-row layout (k_spmv_blk3f,
//    AFEM_MG_F32; the PCG's own product stays fp64), on one rank with the mask
//    fused into the first sweep and the constraint fix into the last (AFEM_MG_FUSE);
//  * coarsest level: dense inverse (<= kDenseMax DoF, symmetric scaling +
//    Cholesky on the host at setup), else 16 Jacobi sweeps;
//  * constraint rows (penalty / eliminated, the PCG's `cons` flags) are taken
//    out of the cycle: z = F V(F r) + C D^-1 r (F free, C constraint masks), so
//    the preconditioner stays SPD and eliminated rows keep a zero direction.
// Several ranks (z-slabs of one box): ONE global V-cycle.  The fine level is
// the slab's owned rows with the system's halo; the coarse levels stay cut
// into z-slabs (owned coarse layer Z = the owner of fine layer 2Z; local
// numbering: owned layers, ghost layer below, ghost layer above; a halo per
// level; the Galerkin rows next to a slab boundary read the neighbour's fine
// boundary rows, exchanged once at setup as 15-entry "fat" rows) down to the
// gather level -- a rank would own no layer, the level fits kDenseMax, or it
// is below 1/512 of the fine grid (AFEM_MG_GATHER) -- whose operator is the
// sum over the ranks of their owned rows' P^T A P parts, replicated with
// everything below it (the one-rank hierarchy, the same arithmetic on every
// rank).  Setup errors are agreed over the ranks (any_rank).
#include "afem_internal.hpp"
#include "kcycle.hpp"

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

namespace afem {

namespace {

inline unsigned grid_for(int64_t n, int threads) { return (unsigned)((n + threads - 1) / threads); }

constexpr int kDenseMax = 512;  // DoF of a coarsest level inverted densely
constexpr int kSweeps = 1;       // pre- and post-smoothing sweeps (C5, n = 128: 1 -> 20 PCG iterations, 43 ms
                                 // per step; 2 -> 16, 55 ms; 3 -> 13, 64 ms)
constexpr int kCoarseSweeps = 16;
constexpr int kPowerIts = 12;

struct Dims {
  int nx, ny, nz;  // cells per axis
  __host__ __device__ int64_t nodes() const { return (int64_t)(nx + 1) * (ny + 1) * (nz + 1); }
  __host__ __device__ int64_t id(int x, int y, int z) const { return x + (int64_t)(nx + 1) * (y + (int64_t)(ny + 1) * z); }
  __host__ __device__ bool in(int x, int y, int z) const
  {
    return x >= 0 && y >= 0 && z >= 0 && x <= nx && y <= ny && z <= nz;
  }
};

// self + the 14 Kuhn edge directions (monotone e in {0,1}^3 \ 0, both signs)
__constant__ int c_st[15][3] = { { 0, 0, 0 },   { 1, 0, 0 },   { 0, 1, 0 },  { 0, 0, 1 },  { 1, 1, 0 },
                                 { 1, 0, 1 },   { 0, 1, 1 },   { 1, 1, 1 },  { -1, 0, 0 }, { 0, -1, 0 },
                                 { 0, 0, -1 },  { -1, -1, 0 }, { -1, 0, -1 }, { 0, -1, -1 }, { -1, -1, -1 } };
const int h_st[15][3] = { { 0, 0, 0 },  { 1, 0, 0 },   { 0, 1, 0 },   { 0, 0, 1 },   { 1, 1, 0 },
                          { 1, 0, 1 },  { 0, 1, 1 },   { 1, 1, 1 },   { -1, 0, 0 },  { 0, -1, 0 },
                          { 0, 0, -1 }, { -1, -1, 0 }, { -1, 0, -1 }, { 0, -1, -1 }, { -1, -1, -1 } };

__device__ __forceinline__ void decompose(const Dims& d, int64_t n, int& x, int& y, int& z)
{
  x = (int)(n % (d.nx + 1));
  const int64_t q = n / (d.nx + 1);
  y = (int)(q % (d.ny + 1));
  z = (int)(q / (d.ny + 1));
}

// A_c = P^T A P, one thread per coarse node row (fixed loop order: deterministic)
template <int K>
__global__ void k_mg_galerkin(Dims fd, Dims cd, const int64_t* __restrict__ fbp, const int32_t* __restrict__ fbc,
                              const double* __restrict__ fv, const int64_t* __restrict__ cbp,
                              const int32_t* __restrict__ cbc, double* __restrict__ cv, int* __restrict__ err)
{
  const int64_t I = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (I >= cd.nodes()) return;
  int cx, cy, cz;
  decompose(cd, I, cx, cy, cz);
  const int64_t c0 = cbp[I];
  const int clen = (int)(cbp[I + 1] - c0);
  for (int o = 0; o < 15; ++o) {
    const int fx = 2 * cx + c_st[o][0], fy = 2 * cy + c_st[o][1], fz = 2 * cz + c_st[o][2];
    if (!fd.in(fx, fy, fz)) continue;
    const double wi = o == 0 ? 1.0 : 0.5;
    const int64_t fi = fd.id(fx, fy, fz);
    const int64_t f0 = fbp[fi];
    const int flen = (int)(fbp[fi + 1] - f0);
    for (int s = 0; s < flen; ++s) {
      int jx, jy, jz;
      decompose(fd, fbc[f0 + s], jx, jy, jz);
      const int a = jx & 1, b = jy & 1, c = jz & 1;
      const int px = jx >> 1, py = jy >> 1, pz = jz >> 1;
      const int np = (a | b | c) ? 2 : 1;
      const double w = wi * (np == 2 ? 0.5 : 1.0);
      for (int p = 0; p < np; ++p) {
        const int32_t J = (int32_t)cd.id(px + p * a, py + p * b, pz + p * c);
        int t = -1;
        for (int q = 0; q < clen; ++q)
          if (cbc[c0 + q] == J) {
            t = q;
            break;
          }
        if (t < 0) {
          *err = 1;
          continue;
        }
        for (int u = 0; u < K; ++u)
          for (int v = 0; v < K; ++v)
            cv[K * K * c0 + K * u * clen + K * t + v] += w * fv[K * K * f0 + K * u * flen + K * s + v];
      }
    }
  }
}

// r_c = P^T r_f
template <int K>
__global__ void k_mg_restrict(Dims fd, Dims cd, const double* __restrict__ rf, double* __restrict__ rc)
{
  const int64_t I = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (I >= cd.nodes()) return;
  int cx, cy, cz;
  decompose(cd, I, cx, cy, cz);
  double acc[K];
  for (int u = 0; u < K; ++u) acc[u] = 0.0;
  for (int o = 0; o < 15; ++o) {
    const int fx = 2 * cx + c_st[o][0], fy = 2 * cy + c_st[o][1], fz = 2 * cz + c_st[o][2];
    if (!fd.in(fx, fy, fz)) continue;
    const double w = o == 0 ? 1.0 : 0.5;
    const int64_t fi = fd.id(fx, fy, fz);
    for (int u = 0; u < K; ++u) acc[u] += w * rf[K * fi + u];
  }
  for (int u = 0; u < K; ++u) rc[K * I + u] = acc[u];
}

// x_f += P x_c
template <int K>
__global__ void k_mg_prolong(Dims fd, Dims cd, const double* __restrict__ xc, double* __restrict__ xf)
{
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= fd.nodes()) return;
  int x, y, z;
  decompose(fd, f, x, y, z);
  const int a = x & 1, b = y & 1, c = z & 1;
  const int64_t P0 = cd.id(x >> 1, y >> 1, z >> 1);
  if (a | b | c) {
    const int64_t P1 = cd.id((x >> 1) + a, (y >> 1) + b, (z >> 1) + c);
    for (int u = 0; u < K; ++u) xf[K * f + u] += 0.5 * (xc[K * P0 + u] + xc[K * P1 + u]);
  }
  else {
    for (int u = 0; u < K; ++u) xf[K * f + u] += xc[K * P0 + u];
  }
}

// point-Jacobi diagonal of a coarse level (its node-diagonal block's diagonal)
template <int K>
__global__ void k_mg_dinv(int64_t n_nodes, const int64_t* __restrict__ bp, const int32_t* __restrict__ bc,
                          const double* __restrict__ v, double* __restrict__ dinv)
{
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_nodes) return;
  const int64_t b0 = bp[r];
  const int len = (int)(bp[r + 1] - b0);
  int s = 0;
  for (int q = 0; q < len; ++q)
    if (bc[b0 + q] == (int32_t)r) s = q;
  for (int u = 0; u < K; ++u) {
    const double d = v[K * K * b0 + K * u * len + K * s + u];
    dinv[K * r + u] = d != 0.0 ? 1.0 / d : 0.0;
  }
}

__global__ void k_mg_scale(int64_t n, double omega, const double* __restrict__ dinv, const double* __restrict__ b,
                           double* __restrict__ x)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] = omega * dinv[i] * b[i];
}

// b = F r and the first sweep from zero x = omega dinv b in one pass (mg_apply's entry)
__global__ void k_mg_mask_scale(int64_t n, const uint8_t* __restrict__ cons, const double* __restrict__ r,
                                double omega, const double* __restrict__ dinv, double* __restrict__ b,
                                double* __restrict__ x)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double bi = cons[i] ? 0.0 : r[i];
    b[i] = bi;
    x[i] = omega * dinv[i] * bi;
  }
}

// F r (constraint rows zeroed)
__global__ void k_mg_mask(int64_t n, const uint8_t* __restrict__ cons, const double* __restrict__ r,
                          double* __restrict__ b)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    b[i] = cons[i] ? 0.0 : r[i];
}

// z = F z + C D^-1 r
__global__ void k_mg_fix(int64_t n, const uint8_t* __restrict__ cons, const double* __restrict__ r,
                         const double* __restrict__ dinv, double* __restrict__ z)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (cons[i]) z[i] = r[i] * dinv[i];
}

__global__ void k_mg_fill(int64_t n, double* __restrict__ v)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    v[i] = 0.5 + (double)(h & 0xFFFF) / 65536.0;
  }
}

// w = dinv .* w, block partials of w.w
__global__ void k_mg_dscale_dot(int64_t n, const double* __restrict__ dinv, double* __restrict__ w,
                                double* __restrict__ partial)
{
  __shared__ double sh[256];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double t = dinv[i] * w[i];
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

// block partials of v.v
__global__ void k_mg_norm2(int64_t n, const double* __restrict__ v, double* __restrict__ partial)
{
  __shared__ double sh[256];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    s += v[i] * v[i];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = sh[0];
}

__global__ void k_mg_mul(int64_t n, double a, double* __restrict__ v)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    v[i] *= a;
}

// x = Ainv b (dense, coarsest level): one wavefront per row, coalesced row reads
__global__ __launch_bounds__(64) void k_mg_gemv(int n, const double* __restrict__ A, const double* __restrict__ b,
                                                double* __restrict__ x)
{
  const int i = blockIdx.x;
  double s = 0.0;
  for (int j = threadIdx.x; j < n; j += 64) s += A[(int64_t)i * n + j] * b[j];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (threadIdx.x == 0) x[i] = s;
}

// fine level of a ghosted slab (block-Jacobi V-cycle): row lengths of the
// owned block (the owned columns are the prefix of each sorted row: ghosts are
// numbered after the owned nodes) and one for every node of the pad layer
__global__ void k_mg_own_len(int64_t nn_own, int64_t nn, const int64_t* __restrict__ bp,
                             const int32_t* __restrict__ bc, int64_t* __restrict__ len)
{
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nn) return;
  if (r >= nn_own) {
    len[r] = 1;
    return;
  }
  int64_t l = 0;
  for (int64_t q = bp[r]; q < bp[r + 1] && bc[q] < nn_own; ++q) ++l;
  len[r] = l;
}
// copy of the owned block (values in the node-block CSR order, K u len + K s + w);
// a pad node gets a decoupled diagonal block: the diagonal of the owned node
// below it (same scale as its neighbours for the smoother and the Galerkin sums)
template <int K>
__global__ void k_mg_own_copy(int64_t nn_own, int64_t nn, int64_t layer, const int64_t* __restrict__ bp,
                              const int32_t* __restrict__ bc, const double* __restrict__ v,
                              const int64_t* __restrict__ nbp, int32_t* __restrict__ nbc, double* __restrict__ nv)
{
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nn) return;
  const int64_t o = nbp[r];
  if (r >= nn_own) {
    const int64_t below = r - layer;
    const int64_t b0 = bp[below];
    const int len = (int)(bp[below + 1] - b0);
    int s = 0;
    for (int q = 0; q < len; ++q)
      if (bc[b0 + q] == (int32_t)below) s = q;
    nbc[o] = (int32_t)r;
    for (int u = 0; u < K; ++u)
      for (int w = 0; w < K; ++w) nv[K * K * o + K * u + w] = u == w ? v[K * K * b0 + K * u * len + K * s + u] : 0.0;
    return;
  }
  const int64_t b0 = bp[r];
  const int len = (int)(bp[r + 1] - b0);
  const int nl = (int)(nbp[r + 1] - o);
  for (int s = 0; s < nl; ++s) nbc[o + s] = bc[b0 + s];
  for (int u = 0; u < K; ++u)
    for (int s = 0; s < nl; ++s)
      for (int w = 0; w < K; ++w) nv[K * K * o + K * u * nl + K * s + w] = v[K * K * b0 + K * u * len + K * s + w];
}
// b = F r on the owned rows, 0 on the pad layer
__global__ void k_mg_mask_pad(int64_t n, int64_t n_all, const uint8_t* __restrict__ cons,
                              const double* __restrict__ r, double* __restrict__ b)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_all; i += (int64_t)gridDim.x * blockDim.x)
    b[i] = i < n && !cons[i] ? r[i] : 0.0;
}

// ---- the global V-cycle over z-slabs: the fine level (and the distributed coarse levels below)
// A slab's local node numbering (Mesh.structured with nranks > 1): the owned
// layers k0 .. k0+nown-1, then the ghost layer below (if any), then the one above.
struct SlabMap {
  int np1;    // nodes per row (nx + 1)
  int64_t L;  // nodes per layer
  int k0, nown, glo;
  int ghi;    // a ghost layer above (distributed coarse levels; level 0 does not use it)
  __host__ __device__ int gz(int li) const { return li < nown ? k0 + li : (li == nown && glo ? k0 - 1 : k0 + nown); }
  __host__ __device__ bool owned_z(int z) const { return z >= k0 && z < k0 + nown; }
  __host__ __device__ bool local_z(int z) const { return owned_z(z) || (glo && z == k0 - 1) || (ghi && z == k0 + nown); }
  __host__ __device__ int local_layer(int z) const { return owned_z(z) ? z - k0 : (z == k0 - 1 ? nown : nown + glo); }
  __host__ __device__ int64_t local_owned(int x, int y, int z) const { return (int64_t)(z - k0) * L + x + (int64_t)np1 * y; }
  __host__ __device__ int64_t local_of(int x, int y, int z) const { return (int64_t)local_layer(z) * L + x + (int64_t)np1 * y; }
  __host__ __device__ int64_t n_local() const { return (int64_t)(nown + glo + ghi) * L; }
};

// the part of A_c = P^T A P over the slab's OWNED fine rows (global coarse
// numbering; summed over the ranks afterwards); loop order of k_mg_galerkin
template <int K>
__global__ void k_mg_galerkin_part(Dims fd, Dims cd, SlabMap sm, const int64_t* __restrict__ fbp,
                                   const int32_t* __restrict__ fbc, const double* __restrict__ fv,
                                   const int64_t* __restrict__ cbp, const int32_t* __restrict__ cbc,
                                   double* __restrict__ cv, int* __restrict__ err)
{
  const int64_t I = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (I >= cd.nodes()) return;
  int cx, cy, cz;
  decompose(cd, I, cx, cy, cz);
  if (2 * cz + 1 < sm.k0 || 2 * cz - 1 >= sm.k0 + sm.nown) return;
  const int64_t c0 = cbp[I];
  const int clen = (int)(cbp[I + 1] - c0);
  for (int o = 0; o < 15; ++o) {
    const int fx = 2 * cx + c_st[o][0], fy = 2 * cy + c_st[o][1], fz = 2 * cz + c_st[o][2];
    if (!fd.in(fx, fy, fz) || !sm.owned_z(fz)) continue;
    const double wi = o == 0 ? 1.0 : 0.5;
    const int64_t fi = sm.local_owned(fx, fy, fz);
    const int64_t f0 = fbp[fi];
    const int flen = (int)(fbp[fi + 1] - f0);
    for (int s = 0; s < flen; ++s) {
      const int64_t col = fbc[f0 + s];
      const int li = (int)(col / sm.L);
      const int64_t pos = col - (int64_t)li * sm.L;
      const int jx = (int)(pos % sm.np1), jy = (int)(pos / sm.np1), jz = sm.gz(li);
      const int a = jx & 1, b = jy & 1, c = jz & 1;
      const int px = jx >> 1, py = jy >> 1, pz = jz >> 1;
      const int np = (a | b | c) ? 2 : 1;
      const double w = wi * (np == 2 ? 0.5 : 1.0);
      for (int p = 0; p < np; ++p) {
        const int32_t J = (int32_t)cd.id(px + p * a, py + p * b, pz + p * c);
        int t = -1;
        for (int q = 0; q < clen; ++q)
          if (cbc[c0 + q] == J) {
            t = q;
            break;
          }
        if (t < 0) {
          *err = 1;
          continue;
        }
        for (int u = 0; u < K; ++u)
          for (int v = 0; v < K; ++v)
            cv[K * K * c0 + K * u * clen + K * t + v] += w * fv[K * K * f0 + K * u * flen + K * s + v];
      }
    }
  }
}

// the part of r_c = P^T r_f over the slab's owned fine nodes (every coarse node
// written: 0 away from the slab; summed over the ranks afterwards)
template <int K>
__global__ void k_mg_restrict_part(Dims fd, Dims cd, SlabMap sm, const double* __restrict__ rf,
                                   double* __restrict__ rc)
{
  const int64_t I = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (I >= cd.nodes()) return;
  int cx, cy, cz;
  decompose(cd, I, cx, cy, cz);
  double acc[K];
  for (int u = 0; u < K; ++u) acc[u] = 0.0;
  if (!(2 * cz + 1 < sm.k0 || 2 * cz - 1 >= sm.k0 + sm.nown)) {
    for (int o = 0; o < 15; ++o) {
      const int fx = 2 * cx + c_st[o][0], fy = 2 * cy + c_st[o][1], fz = 2 * cz + c_st[o][2];
      if (!fd.in(fx, fy, fz) || !sm.owned_z(fz)) continue;
      const double w = o == 0 ? 1.0 : 0.5;
      const int64_t fi = sm.local_owned(fx, fy, fz);
      for (int u = 0; u < K; ++u) acc[u] += w * rf[K * fi + u];
    }
  }
  for (int u = 0; u < K; ++u) rc[K * I + u] = acc[u];
}

// x_f += P x_c on the slab's owned fine nodes (x_c global)
template <int K>
__global__ void k_mg_prolong_own(Dims cd, SlabMap sm, int64_t nn_own, const double* __restrict__ xc,
                                 double* __restrict__ xf)
{
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= nn_own) return;
  const int li = (int)(f / sm.L);
  const int64_t pos = f - (int64_t)li * sm.L;
  const int x = (int)(pos % sm.np1), y = (int)(pos / sm.np1), z = sm.k0 + li;
  const int a = x & 1, b = y & 1, c = z & 1;
  const int64_t P0 = cd.id(x >> 1, y >> 1, z >> 1);
  if (a | b | c) {
    const int64_t P1 = cd.id((x >> 1) + a, (y >> 1) + b, (z >> 1) + c);
    for (int u = 0; u < K; ++u) xf[K * f + u] += 0.5 * (xc[K * P0 + u] + xc[K * P1 + u]);
  }
  else {
    for (int u = 0; u < K; ++u) xf[K * f + u] += xc[K * P0 + u];
  }
}

// ---- distributed coarse levels: every level above the gather level is cut into
// z-slabs like the fine one (owned coarse layer Z = the owner of fine layer 2Z),
// local numbering as level 0 (owned layers, ghost layer below, ghost layer above),
// one halo per level.  The Galerkin product of an owned coarse row needs the fine
// rows of the layers 2Z - 1 .. 2Z + 1, so the fine boundary layers' rows travel
// to the neighbours once at setup, as "fat" rows: 15 entries of (global column
// id, K^2 values), column -1 past the row's end.  Fat slots: the first and the
// last owned layer (sent), the ghost layer below and the one above (received).
constexpr int kFatRow = 15;

__host__ __device__ inline int fat_slot(const SlabMap& sm, int li)
{
  if (li == 0) return 0;
  if (li == sm.nown - 1) return 1;
  return li == sm.nown && sm.glo ? 2 : 3;
}

template <int K>
__global__ void k_mg_fat_rows(Dims gd, SlabMap sm, const int64_t* __restrict__ bp, const int32_t* __restrict__ bc,
                              const double* __restrict__ v, double* __restrict__ fat, int* __restrict__ err)
{
  constexpr int E = 1 + K * K;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2 * sm.L) return;
  const int li = t < sm.L ? 0 : sm.nown - 1;
  if (t >= sm.L && sm.nown == 1) return;  // one owned layer: slot 0 only
  const int64_t r = (int64_t)li * sm.L + t % sm.L;
  const int64_t b0 = bp[r];
  const int len = (int)(bp[r + 1] - b0);
  if (len > kFatRow) *err = 1;
  double* out = fat + ((int64_t)fat_slot(sm, li) * sm.L + t % sm.L) * kFatRow * E;
  for (int s = 0; s < kFatRow; ++s) {
    if (s < len) {
      const int64_t col = bc[b0 + s];
      const int lc = (int)(col / sm.L);
      const int64_t pos = col - (int64_t)lc * sm.L;
      out[s * E] = (double)gd.id((int)(pos % sm.np1), (int)(pos / sm.np1), sm.gz(lc));
      for (int u = 0; u < K; ++u)
        for (int w = 0; w < K; ++w) out[s * E + 1 + K * u + w] = v[K * K * b0 + K * u * len + K * s + w];
    }
    else {
      out[s * E] = -1.0;
    }
  }
}

// A_c = P^T A P for the OWNED rows of a distributed coarse level (local
// numbering, loop order of k_mg_galerkin); fine rows of ghost layers from `fat`
template <int K>
__global__ void k_mg_galerkin_dist(Dims fgd, Dims cgd, SlabMap fsm, SlabMap csm, const int64_t* __restrict__ fbp,
                                   const int32_t* __restrict__ fbc, const double* __restrict__ fv,
                                   const double* __restrict__ fat, const int64_t* __restrict__ cbp,
                                   const int32_t* __restrict__ cbc, double* __restrict__ cv, int* __restrict__ err)
{
  constexpr int E = 1 + K * K;
  const int64_t I = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (I >= (int64_t)csm.nown * csm.L) return;
  const int li = (int)(I / csm.L);
  const int64_t pos = I - (int64_t)li * csm.L;
  const int cx = (int)(pos % csm.np1), cy = (int)(pos / csm.np1), cz = csm.k0 + li;
  const int64_t c0 = cbp[I];
  const int clen = (int)(cbp[I + 1] - c0);
  for (int o = 0; o < 15; ++o) {
    const int fx = 2 * cx + c_st[o][0], fy = 2 * cy + c_st[o][1], fz = 2 * cz + c_st[o][2];
    if (!fgd.in(fx, fy, fz)) continue;
    if (!fsm.local_z(fz)) {
      *err = 1;
      continue;
    }
    const double wi = o == 0 ? 1.0 : 0.5;
    const bool own = fsm.owned_z(fz);
    const int64_t fi = fsm.local_of(fx, fy, fz);
    int64_t f0 = 0;
    int flen = 0;
    const double* fr = nullptr;
    if (own) {
      f0 = fbp[fi];
      flen = (int)(fbp[fi + 1] - f0);
    }
    else {
      fr = fat + ((int64_t)fat_slot(fsm, fsm.local_layer(fz)) * fsm.L + fx + (int64_t)fsm.np1 * fy) * kFatRow * E;
      while (flen < kFatRow && fr[flen * E] >= 0.0) ++flen;
    }
    for (int s = 0; s < flen; ++s) {
      int jx, jy, jz;
      if (own) {
        const int64_t col = fbc[f0 + s];
        const int lc = (int)(col / fsm.L);
        const int64_t p = col - (int64_t)lc * fsm.L;
        jx = (int)(p % fsm.np1);
        jy = (int)(p / fsm.np1);
        jz = fsm.gz(lc);
      }
      else {
        decompose(fgd, (int64_t)fr[s * E], jx, jy, jz);
      }
      const int a = jx & 1, b = jy & 1, c = jz & 1;
      const int px = jx >> 1, py = jy >> 1, pz = jz >> 1;
      const int np = (a | b | c) ? 2 : 1;
      const double w = wi * (np == 2 ? 0.5 : 1.0);
      for (int p = 0; p < np; ++p) {
        const int qz = pz + p * c;
        if (!csm.local_z(qz)) {
          *err = 1;
          continue;
        }
        const int32_t J = (int32_t)csm.local_of(px + p * a, py + p * b, qz);
        int t = -1;
        for (int q = 0; q < clen; ++q)
          if (cbc[c0 + q] == J) {
            t = q;
            break;
          }
        if (t < 0) {
          *err = 1;
          continue;
        }
        for (int u = 0; u < K; ++u)
          for (int v = 0; v < K; ++v)
            cv[K * K * c0 + K * u * clen + K * t + v] +=
            w * (own ? fv[K * K * f0 + K * u * flen + K * s + v] : fr[s * E + 1 + K * u + v]);
      }
    }
  }
}

// r_c = P^T r_f on the owned coarse nodes (r_f with its ghost layers exchanged)
template <int K>
__global__ void k_mg_restrict_dist(Dims fgd, SlabMap fsm, SlabMap csm, const double* __restrict__ rf,
                                   double* __restrict__ rc)
{
  const int64_t I = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (I >= (int64_t)csm.nown * csm.L) return;
  const int li = (int)(I / csm.L);
  const int64_t pos = I - (int64_t)li * csm.L;
  const int cx = (int)(pos % csm.np1), cy = (int)(pos / csm.np1), cz = csm.k0 + li;
  double acc[K];
  for (int u = 0; u < K; ++u) acc[u] = 0.0;
  for (int o = 0; o < 15; ++o) {
    const int fx = 2 * cx + c_st[o][0], fy = 2 * cy + c_st[o][1], fz = 2 * cz + c_st[o][2];
    if (!fgd.in(fx, fy, fz)) continue;
    const double w = o == 0 ? 1.0 : 0.5;
    const int64_t fi = fsm.local_of(fx, fy, fz);
    for (int u = 0; u < K; ++u) acc[u] += w * rf[K * fi + u];
  }
  for (int u = 0; u < K; ++u) rc[K * I + u] = acc[u];
}

// x_f += P x_c on the owned fine nodes (x_c with its ghost layers exchanged)
template <int K>
__global__ void k_mg_prolong_dist(SlabMap fsm, SlabMap csm, const double* __restrict__ xc, double* __restrict__ xf)
{
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= (int64_t)fsm.nown * fsm.L) return;
  const int li = (int)(f / fsm.L);
  const int64_t pos = f - (int64_t)li * fsm.L;
  const int x = (int)(pos % fsm.np1), y = (int)(pos / fsm.np1), z = fsm.k0 + li;
  const int a = x & 1, b = y & 1, c = z & 1;
  const int64_t P0 = csm.local_of(x >> 1, y >> 1, z >> 1);
  if (a | b | c) {
    const int64_t P1 = csm.local_of((x >> 1) + a, (y >> 1) + b, (z >> 1) + c);
    for (int u = 0; u < K; ++u) xf[K * f + u] += 0.5 * (xc[K * P0 + u] + xc[K * P1 + u]);
  }
  else {
    for (int u = 0; u < K; ++u) xf[K * f + u] += xc[K * P0 + u];
  }
}

// the power iteration's start vector by GLOBAL index (the one-rank sequence of k_mg_fill)
__global__ void k_mg_fill_off(int64_t n, int64_t off, double* __restrict__ v)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t h = (uint64_t)(i + off) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    v[i] = 0.5 + (double)(h & 0xFFFF) / 65536.0;
  }
}

constexpr int kVec = 1024;  // grid of the vector kernels

}  // namespace

struct MgLevel {
  Dims d{};
  int64_t nn = 0, n = 0;  // nodes, scalar rows (k * nodes)
  const int64_t* bp = nullptr;
  const int32_t* bc = nullptr;
  const double* v = nullptr;
  const double* dinv = nullptr;
  DevBuf<int64_t> own_bp;
  DevBuf<int32_t> own_bc;
  DevBuf<double> own_v, own_dinv;
  DevBuf<double> x, t, b, r;  // iterate (ping-pong x / t), right-hand side, residual
  DevBuf<float> v32;          // AFEM_MG_F32: the values in k_spmv_blk3f's layout (block-3 levels)
  DevBuf<double> kc1, kv1, krt, kcoef;  // K-cycle level (AFEM_MG_KCYCLE)
  double omega = 0.0;
  // a distributed level (global V-cycle over z-slabs): the slab's owned rows in
  // local numbering (sm), the global box gd, the halo of its vectors (level 0:
  // the system's own), vectors x / t / r with the ghost entries (ncol)
  bool dist = false;
  SlabMap sm{};
  Dims gd{};
  std::unique_ptr<Halo> halo;
  int64_t ncol = 0;
  std::vector<int> lo, hi;  // every rank's owned layers [lo, hi) at this level
};

struct Multigrid {
  int k = 1;
  int sweeps = kSweeps;
  // global V-cycle over z-slabs: level 0 is the slab's owned rows (vectors with
  // the ghost entries of the system's halo), levels >= 1 the global box's
  bool global = false;
  SlabMap sm{};
  Dims gfine{};
  int n_dist = 0;  // levels [0, n_dist) are distributed, the rest replicated
  std::vector<MgLevel> lv;
  DevBuf<double> ainv;  // dense inverse of the coarsest level (n_dense x n_dense) or empty
  int n_dense = 0;
  DevBuf<double> partial;
  // reuse key (multigrid = 2): the fine structure the hierarchy was built for
  const void* key_rows = nullptr;
  const void* key_vals = nullptr;
  int64_t key_n = 0;
};

void MgDeleter::operator()(Multigrid* m) const { delete m; }

namespace {
// one global V-cycle over the slabs (else: block-Jacobi V-cycles on the owned blocks)
bool mg_global_mode(const LinearSystem& ls)
{
  if (!ls.mg_multi || !ls.halo || !ls.halo->comm) return false;
  const char* e = variant("AFEM_MG_MULTI");
  if (e && std::string(e) == "block") return false;
  return ls.mg_nx >= 2 && ls.mg_nx % 2 == 0 && ls.mg_nzg >= 2 && ls.mg_nzg % 2 == 0 && ls.mg_nz >= 0;
}
}  // namespace

bool mg_available(const LinearSystem& ls)
{
  if (ls.mg_k >= 1 && ls.mg_k <= 3 && mg_global_mode(ls)) {
    const Dims d{ ls.mg_nx, ls.mg_nx, ls.mg_nz };
    if (d.nodes() * ls.mg_k != ls.n_rows) return false;
    return ls.mg_k == 1 ? ls.csr_rows != nullptr : (ls.blk_k == ls.mg_k && ls.blk_rows);
  }
  if (ls.mg_k < 1 || ls.mg_k > 3 || ls.mg_nx < 2 || ls.mg_nz < 1) return false;
  if (ls.mg_nx % 2) return false;                      // no coarse level
  if (!ls.mg_multi && ls.mg_nz % 2) return false;      // one rank: an odd box has no coarse level
  if (ls.mg_nz + ls.mg_nz % 2 < 2) return false;
  if (ls.halo && !ls.mg_multi) return false;           // a halo over a mesh whose owned part is no box
  const Dims d{ ls.mg_nx, ls.mg_nx, ls.mg_nz };
  if (d.nodes() * ls.mg_k != ls.n_rows) return false;
  if (ls.mg_k == 1 ? !ls.csr_rows : (ls.blk_k != ls.mg_k || !ls.blk_rows)) return false;
  return true;
}

int mg_levels(const LinearSystem& ls) { return ls.mg ? (int)ls.mg->lv.size() : 0; }

namespace {

template <class F>
void dispatch_k(int k, F&& f)
{
  if (k == 3) f(std::integral_constant<int, 3>{});
  else if (k == 2) f(std::integral_constant<int, 2>{});
  else f(std::integral_constant<int, 1>{});
}

void coarse_structure(const Dims& d, std::vector<int64_t>& bp, std::vector<int32_t>& bc)
{
  const int64_t n = d.nodes();
  bp.assign(n + 1, 0);
  bc.clear();
  bc.reserve(n * 15);
  std::vector<int32_t> row;
  for (int z = 0; z <= d.nz; ++z)
    for (int y = 0; y <= d.ny; ++y)
      for (int x = 0; x <= d.nx; ++x) {
        row.clear();
        for (int o = 0; o < 15; ++o) {
          const int X = x + h_st[o][0], Y = y + h_st[o][1], Z = z + h_st[o][2];
          if (d.in(X, Y, Z)) row.push_back((int32_t)d.id(X, Y, Z));
        }
        std::sort(row.begin(), row.end());
        bc.insert(bc.end(), row.begin(), row.end());
        bp[d.id(x, y, z) + 1] = (int64_t)bc.size();
      }
}

double host_sum(Ctx& ctx, const DevBuf<double>& partial, int n)
{
  std::vector<double> h(n);
  AFEM_HIP(hipMemcpyAsync(h.data(), partial.p, n * sizeof(double), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  double s = 0.0;
  for (double v : h) s += v;
  return s;
}

// lambda_max(D^-1 A) by power iteration (x, t as work vectors)
double power_lambda(Ctx& ctx, Multigrid& mg, MgLevel& L)
{
  const int k = mg.k;
  const unsigned g = (unsigned)std::min<int64_t>(kVec, (L.n + 255) / 256);
  hipLaunchKernelGGL(k_mg_fill, dim3(g), dim3(256), 0, ctx.stream, L.n, L.x.p);
  AFEM_LAUNCHED();
  double lam = 0.0, nv = 0.0;
  hipLaunchKernelGGL(k_mg_norm2, dim3(g), dim3(256), 0, ctx.stream, L.n, L.x.p, mg.partial.p);
  AFEM_LAUNCHED();
  nv = std::sqrt(host_sum(ctx, mg.partial, (int)g));
  for (int it = 0; it < kPowerIts; ++it) {
    spmv_blk_epi(ctx, k, 0, L.nn, L.bp, L.bc, L.v, L.x.p, L.t.p, nullptr, nullptr, 0.0);
    hipLaunchKernelGGL(k_mg_dscale_dot, dim3(g), dim3(256), 0, ctx.stream, L.n, L.dinv, L.t.p, mg.partial.p);
    AFEM_LAUNCHED();
    const double nw = std::sqrt(host_sum(ctx, mg.partial, (int)g));
    lam = nv > 0 ? nw / nv : 0.0;
    if (!(nw > 0)) break;
    hipLaunchKernelGGL(k_mg_mul, dim3(g), dim3(256), 0, ctx.stream, L.n, 1.0 / nw, L.t.p);
    AFEM_LAUNCHED();
    std::swap(L.x, L.t);
    nv = 1.0;
  }
  return lam;
}

// dense inverse of the coarsest operator: symmetric diagonal scaling, Cholesky,
// inverse (host; <= kDenseMax DoF)
bool dense_inverse(Ctx& ctx, Multigrid& mg, MgLevel& L)
{
  const int k = mg.k;
  const int m = (int)L.n;
  std::vector<int64_t> bp(L.nn + 1);
  AFEM_HIP(hipMemcpyAsync(bp.data(), L.bp, (L.nn + 1) * 8, hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  const int64_t nb = bp[L.nn];
  std::vector<int32_t> bc(nb);
  std::vector<double> v((size_t)nb * k * k);
  AFEM_HIP(hipMemcpyAsync(bc.data(), L.bc, nb * 4, hipMemcpyDeviceToHost, ctx.stream));
  AFEM_HIP(hipMemcpyAsync(v.data(), L.v, v.size() * 8, hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  std::vector<double> A((size_t)m * m, 0.0);
  for (int64_t r = 0; r < L.nn; ++r) {
    const int len = (int)(bp[r + 1] - bp[r]);
    for (int s = 0; s < len; ++s)
      for (int u = 0; u < k; ++u)
        for (int w = 0; w < k; ++w)
          A[(size_t)(k * r + u) * m + k * bc[bp[r] + s] + w] = v[k * k * bp[r] + k * u * len + k * s + w];
  }
  std::vector<double> sc(m);
  for (int i = 0; i < m; ++i) {
    if (!(A[(size_t)i * m + i] > 0)) return false;
    sc[i] = 1.0 / std::sqrt(A[(size_t)i * m + i]);
  }
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < m; ++j) A[(size_t)i * m + j] *= sc[i] * sc[j];
  // Cholesky A = L L^T (lower, in place)
  for (int j = 0; j < m; ++j) {
    double d = A[(size_t)j * m + j];
    for (int q = 0; q < j; ++q) d -= A[(size_t)j * m + q] * A[(size_t)j * m + q];
    if (!(d > 0)) return false;
    d = std::sqrt(d);
    A[(size_t)j * m + j] = d;
    for (int i = j + 1; i < m; ++i) {
      double s = A[(size_t)i * m + j];
      for (int q = 0; q < j; ++q) s -= A[(size_t)i * m + q] * A[(size_t)j * m + q];
      A[(size_t)i * m + j] = s / d;
    }
  }
  // inverse column by column: solve L L^T x = e_c
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
  mg.ainv.alloc((size_t)m * m);
  AFEM_HIP(hipMemcpyAsync(mg.ainv.p, inv.data(), inv.size() * 8, hipMemcpyHostToDevice, ctx.stream));
  ctx.sync();
  mg.n_dense = m;
  return true;
}

double allreduce_scalar(LinearSystem& ls, double v)
{
  Ctx& ctx = *ls.ctx;
  DevBuf<double> d;
  d.alloc(1);
  AFEM_HIP(hipMemcpyAsync(d.p, &v, sizeof(double), hipMemcpyHostToDevice, ctx.stream));
  comm_allreduce(ls.halo->comm, ctx, d.p, 1);
  double out = 0.0;
  AFEM_HIP(hipMemcpyAsync(&out, d.p, sizeof(double), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  return out;
}

// lambda_max(D^-1 A) of the distributed fine level: the one-rank power
// iteration with the halo exchanged before every product and the norms summed
// over the ranks (start vector by global index)
Halo& level_halo(LinearSystem& ls, MgLevel& L) { return L.halo ? *L.halo : *ls.halo; }

double power_lambda_global(LinearSystem& ls, Multigrid& mg, MgLevel& L)
{
  Ctx& ctx = *ls.ctx;
  const int k = mg.k;
  Halo& H = level_halo(ls, L);
  const unsigned g = (unsigned)std::min<int64_t>(kVec, (L.n + 255) / 256);
  hipLaunchKernelGGL(k_mg_fill_off, dim3(g), dim3(256), 0, ctx.stream, L.n, (int64_t)k * L.sm.k0 * L.sm.L, L.x.p);
  AFEM_LAUNCHED();
  hipLaunchKernelGGL(k_mg_norm2, dim3(g), dim3(256), 0, ctx.stream, L.n, L.x.p, mg.partial.p);
  AFEM_LAUNCHED();
  double nv = std::sqrt(allreduce_scalar(ls, host_sum(ctx, mg.partial, (int)g)));
  double lam = 0.0;
  for (int it = 0; it < kPowerIts; ++it) {
    halo_exchange(H, ctx, L.x.p);
    spmv_blk_epi(ctx, k, 0, L.nn, L.bp, L.bc, L.v, L.x.p, L.t.p, nullptr, nullptr, 0.0);
    hipLaunchKernelGGL(k_mg_dscale_dot, dim3(g), dim3(256), 0, ctx.stream, L.n, L.dinv, L.t.p, mg.partial.p);
    AFEM_LAUNCHED();
    const double nw = std::sqrt(allreduce_scalar(ls, host_sum(ctx, mg.partial, (int)g)));
    lam = nv > 0 ? nw / nv : 0.0;
    if (!(nw > 0)) break;
    hipLaunchKernelGGL(k_mg_mul, dim3(g), dim3(256), 0, ctx.stream, L.n, 1.0 / nw, L.t.p);
    AFEM_LAUNCHED();
    std::swap(L.x, L.t);
    nv = 1.0;
  }
  return lam;
}

// the halo of a distributed level's vectors: its owned boundary layers to the
// z-neighbours, their layers into its ghost layers (node ids x `width`, slots
// of `slot`: the vector's layer of a local layer; identity for plain vectors)
template <class Slot>
std::unique_ptr<Halo> slab_halo(LinearSystem& ls, const SlabMap& sm, int width, Slot slot)
{
  Ctx& ctx = *ls.ctx;
  Comm* comm = ls.halo->comm;
  const int rank = comm_rank(comm);
  std::vector<int32_t> nbr, si, ri;
  std::vector<int64_t> sc, rc;
  auto layer = [&](int li, std::vector<int32_t>& out) {
    for (int64_t i = 0; i < sm.L; ++i) out.push_back((int32_t)(slot(li) * sm.L + i));
  };
  if (sm.glo) {
    nbr.push_back(rank - 1);
    sc.push_back(sm.L);
    rc.push_back(sm.L);
    layer(0, si);
    layer(sm.nown, ri);
  }
  if (sm.ghi) {
    nbr.push_back(rank + 1);
    sc.push_back(sm.L);
    rc.push_back(sm.L);
    layer(sm.nown - 1, si);
    layer(sm.nown + sm.glo, ri);
  }
  expand_dof_lists(width, sc, rc, si, ri);
  std::unique_ptr<Halo> h(new Halo());
  halo_setup(*h, ctx, comm, (int)nbr.size(), nbr.data(), sc.data(), si.data(), rc.data(), ri.data());
  return h;
}

// every rank's owned layers of a distributed level (summed over the ranks)
void gather_ranges(LinearSystem& ls, MgLevel& L)
{
  Ctx& ctx = *ls.ctx;
  Comm* comm = ls.halo->comm;
  const int nr = comm_nranks(comm), rank = comm_rank(comm);
  std::vector<double> h(2 * nr, 0.0);
  h[2 * rank] = L.sm.k0;
  h[2 * rank + 1] = L.sm.k0 + L.sm.nown;
  DevBuf<double> d;
  d.alloc(h.size());
  AFEM_HIP(hipMemcpyAsync(d.p, h.data(), h.size() * 8, hipMemcpyHostToDevice, ctx.stream));
  comm_allreduce(comm, ctx, d.p, (int64_t)h.size());
  AFEM_HIP(hipMemcpyAsync(h.data(), d.p, h.size() * 8, hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  L.lo.resize(nr);
  L.hi.resize(nr);
  for (int r = 0; r < nr; ++r) {
    L.lo[r] = (int)h[2 * r];
    L.hi[r] = (int)h[2 * r + 1];
  }
}

// the error flag of a setup step, the same on every rank (a rank
// that failed alone would leave the others waiting in a collective)
bool any_rank(LinearSystem& ls, const DevBuf<int>& err)
{
  int h = 0;
  AFEM_HIP(hipMemcpyAsync(&h, err.p, sizeof(int), hipMemcpyDeviceToHost, ls.ctx->stream));
  ls.ctx->sync();
  return allreduce_scalar(ls, h ? 1.0 : 0.0) > 0.0;
}

// a distributed coarse level from the distributed level F: owned coarse layer Z
// = the rank owning fine layer 2Z; Galerkin rows on the owned coarse nodes
MgLevel dist_coarse(LinearSystem& ls, Multigrid& mg, MgLevel& F, const Dims& cgd, const std::vector<int>& clo,
                    const std::vector<int>& chi)
{
  Ctx& ctx = *ls.ctx;
  const int k = mg.k;
  const int rank = comm_rank(ls.halo->comm);
  MgLevel C;
  C.dist = true;
  C.gd = cgd;
  C.lo = clo;
  C.hi = chi;
  C.sm = SlabMap{ cgd.nx + 1, (int64_t)(cgd.nx + 1) * (cgd.ny + 1), clo[rank], chi[rank] - clo[rank],
                  clo[rank] > 0 ? 1 : 0, chi[rank] <= cgd.nz ? 1 : 0 };
  C.d = Dims{ cgd.nx, cgd.ny, C.sm.nown - 1 };
  C.nn = (int64_t)C.sm.nown * C.sm.L;
  C.n = k * C.nn;
  C.ncol = k * C.sm.n_local();
  // owned rows: the coarse 15-block Kuhn stencil, local column ids, sorted
  std::vector<int64_t> hbp(C.nn + 1, 0);
  std::vector<int32_t> hbc;
  hbc.reserve(C.nn * 15);
  std::vector<int32_t> row;
  for (int64_t I = 0; I < C.nn; ++I) {
    const int li = (int)(I / C.sm.L);
    const int64_t pos = I - (int64_t)li * C.sm.L;
    const int x = (int)(pos % C.sm.np1), y = (int)(pos / C.sm.np1), z = C.sm.k0 + li;
    row.clear();
    for (int o = 0; o < 15; ++o) {
      const int X = x + h_st[o][0], Y = y + h_st[o][1], Z = z + h_st[o][2];
      if (cgd.in(X, Y, Z)) row.push_back((int32_t)C.sm.local_of(X, Y, Z));
    }
    std::sort(row.begin(), row.end());
    hbc.insert(hbc.end(), row.begin(), row.end());
    hbp[I + 1] = (int64_t)hbc.size();
  }
  C.own_bp.alloc(hbp.size());
  C.own_bc.alloc(hbc.size());
  AFEM_HIP(hipMemcpyAsync(C.own_bp.p, hbp.data(), hbp.size() * 8, hipMemcpyHostToDevice, ctx.stream));
  AFEM_HIP(hipMemcpyAsync(C.own_bc.p, hbc.data(), hbc.size() * 4, hipMemcpyHostToDevice, ctx.stream));
  C.own_v.alloc(hbc.size() * k * k);
  AFEM_HIP(hipMemsetAsync(C.own_v.p, 0, C.own_v.bytes(), ctx.stream));
  C.own_dinv.alloc(C.n);
  // the fine boundary layers' rows to the neighbours (fat rows)
  const int W = kFatRow * (1 + k * k);
  DevBuf<double> fat;
  fat.alloc((size_t)4 * F.sm.L * W);
  DevBuf<int> err;
  err.alloc(1);
  AFEM_HIP(hipMemsetAsync(err.p, 0, sizeof(int), ctx.stream));
  dispatch_k(k, [&](auto kc) {
    constexpr int K = decltype(kc)::value;
    hipLaunchKernelGGL(k_mg_fat_rows<K>, dim3(grid_for(2 * F.sm.L, 128)), dim3(128), 0, ctx.stream, F.gd, F.sm, F.bp,
                       F.bc, F.v, fat.p, err.p);
    AFEM_LAUNCHED();
  });
  const SlabMap fsm = F.sm;
  auto fat_halo = slab_halo(ls, fsm, W, [&](int li) { return fat_slot(fsm, li); });
  halo_exchange(*fat_halo, ctx, fat.p);
  dispatch_k(k, [&](auto kc) {
    constexpr int K = decltype(kc)::value;
    const unsigned g = (unsigned)grid_for(C.nn, 128);
    hipLaunchKernelGGL(k_mg_galerkin_dist<K>, dim3(g), dim3(128), 0, ctx.stream, F.gd, cgd, F.sm, C.sm, F.bp, F.bc,
                       F.v, fat.p, C.own_bp.p, C.own_bc.p, C.own_v.p, err.p);
    AFEM_LAUNCHED();
    hipLaunchKernelGGL(k_mg_dinv<K>, dim3(g), dim3(128), 0, ctx.stream, C.nn, C.own_bp.p, C.own_bc.p, C.own_v.p,
                       C.own_dinv.p);
    AFEM_LAUNCHED();
  });
  AFEM_REQUIRE(!any_rank(ls, err), AFEM_ERR_STATE, "multigrid: distributed Galerkin product outside the coarse stencil");
  C.bp = C.own_bp.p;
  C.bc = C.own_bc.p;
  C.v = C.own_v.p;
  C.dinv = C.own_dinv.p;
  C.halo = slab_halo(ls, C.sm, k, [](int li) { return li; });
  return C;
}

// the first replicated level (the global coarse box) from the distributed level
// F: A_c = sum over the ranks of their owned rows' P^T A P parts
MgLevel gathered_coarse(LinearSystem& ls, Multigrid& mg, MgLevel& F)
{
  Ctx& ctx = *ls.ctx;
  const int k = mg.k;
  MgLevel C;
  C.d = Dims{ F.gd.nx / 2, F.gd.ny / 2, F.gd.nz / 2 };
  C.nn = C.d.nodes();
  C.n = k * C.nn;
  std::vector<int64_t> hbp;
  std::vector<int32_t> hbc;
  coarse_structure(C.d, hbp, hbc);
  C.own_bp.alloc(hbp.size());
  C.own_bc.alloc(hbc.size());
  AFEM_HIP(hipMemcpyAsync(C.own_bp.p, hbp.data(), hbp.size() * 8, hipMemcpyHostToDevice, ctx.stream));
  AFEM_HIP(hipMemcpyAsync(C.own_bc.p, hbc.data(), hbc.size() * 4, hipMemcpyHostToDevice, ctx.stream));
  C.own_v.alloc(hbc.size() * k * k);
  AFEM_HIP(hipMemsetAsync(C.own_v.p, 0, C.own_v.bytes(), ctx.stream));
  C.own_dinv.alloc(C.n);
  DevBuf<int> err;
  err.alloc(1);
  AFEM_HIP(hipMemsetAsync(err.p, 0, sizeof(int), ctx.stream));
  const unsigned g = (unsigned)grid_for(C.nn, 128);
  dispatch_k(k, [&](auto kc) {
    constexpr int K = decltype(kc)::value;
    hipLaunchKernelGGL(k_mg_galerkin_part<K>, dim3(g), dim3(128), 0, ctx.stream, F.gd, C.d, F.sm, F.bp, F.bc, F.v,
                       C.own_bp.p, C.own_bc.p, C.own_v.p, err.p);
    AFEM_LAUNCHED();
  });
  AFEM_REQUIRE(!any_rank(ls, err), AFEM_ERR_STATE, "multigrid: Galerkin product outside the coarse Kuhn stencil");
  comm_allreduce(ls.halo->comm, ctx, C.own_v.p, (int64_t)C.own_v.n);
  dispatch_k(k, [&](auto kc) {
    constexpr int K = decltype(kc)::value;
    hipLaunchKernelGGL(k_mg_dinv<K>, dim3(g), dim3(128), 0, ctx.stream, C.nn, C.own_bp.p, C.own_bc.p, C.own_v.p,
                       C.own_dinv.p);
    AFEM_LAUNCHED();
  });
  C.bp = C.own_bp.p;
  C.bc = C.own_bc.p;
  C.v = C.own_v.p;
  C.dinv = C.own_dinv.p;
  ctx.sync();
  return C;
}

}  // namespace

void mg_setup(LinearSystem& ls)
{
  Ctx& ctx = *ls.ctx;
  AFEM_REQUIRE(mg_available(ls), AFEM_ERR_STATE, "multigrid: not a structured box / z-slab system");
  const bool reuse = ls.opts.multigrid == 2;
  const void* krows = ls.mg_k == 1 ? (const void*)ls.csr_rows : (const void*)ls.blk_rows;
  if (reuse && ls.mg && ls.mg->key_rows == krows && ls.mg->key_vals == ls.csr_vals && ls.mg->key_n == ls.n_rows) {
    // the fine products follow the live values (re-assembled in place every C5 step), as the fp64 ones do
    MgLevel& L0 = ls.mg->lv[0];
    if (L0.v32.p) blk3_to_f32(ctx, L0.nn, L0.bp, L0.v, L0.v32.p);
    return;
  }
  auto mg = std::unique_ptr<Multigrid, MgDeleter>(new Multigrid());
  const int k = ls.mg_k;
  mg->k = k;
  mg->partial.alloc(kVec);
  mg->global = mg_global_mode(ls);
  DevBuf<int> err;
  err.alloc(1);
  AFEM_HIP(hipMemsetAsync(err.p, 0, sizeof(int), ctx.stream));
  {
    MgLevel L;
    const int64_t* bp = k == 1 ? ls.csr_rows : ls.blk_rows;
    const int32_t* bc = k == 1 ? ls.csr_cols : ls.blk_cols;
    if (mg->global) {
      // level 0: the slab's owned rows as they are (local columns, ghosts included)
      L.d = Dims{ ls.mg_nx, ls.mg_nx, ls.mg_nz };
      L.nn = L.d.nodes();
      L.n = k * L.nn;
      L.bp = bp;
      L.bc = bc;
      L.v = ls.csr_vals;
      L.dinv = ls.dinv.p;
      mg->sm = SlabMap{ ls.mg_nx + 1, (int64_t)(ls.mg_nx + 1) * (ls.mg_nx + 1), ls.mg_k0, ls.mg_nz + 1,
                        ls.mg_glo ? 1 : 0, ls.mg_k0 + ls.mg_nz + 1 <= ls.mg_nzg ? 1 : 0 };
      mg->gfine = Dims{ ls.mg_nx, ls.mg_nx, ls.mg_nzg };
      L.dist = true;
      L.sm = mg->sm;
      L.gd = mg->gfine;
      L.ncol = ls.n_cols;
      gather_ranges(ls, L);
      mg->lv.push_back(std::move(L));
      mg->n_dist = 1;
      // distributed coarse levels while every rank keeps a layer and the level is
      // above 1/AFEM_MG_GATHER of the fine grid (default 512), then the global
      // coarse box, replicated (the one-rank hierarchy's levels either way)
      const char* ge = variant("AFEM_MG_GATHER");
      const double ratio = ge && *ge ? std::atof(ge) : 512.0;
      while (true) {
        MgLevel& F = mg->lv.back();
        const bool coarsen = (int64_t)k * F.gd.nodes() > kDenseMax && F.gd.nx % 2 == 0 && F.gd.ny % 2 == 0 &&
                             F.gd.nz % 2 == 0 && F.gd.nx >= 2 && F.gd.nz >= 2;
        if (!coarsen) break;  // F is the coarsest level: smoothing only
        const Dims cgd{ F.gd.nx / 2, F.gd.ny / 2, F.gd.nz / 2 };
        std::vector<int> clo(F.lo.size()), chi(F.lo.size());
        bool every = true;
        for (size_t r = 0; r < F.lo.size(); ++r) {
          clo[r] = (F.lo[r] + 1) / 2;
          chi[r] = (F.hi[r] + 1) / 2;
          every = every && chi[r] > clo[r];
        }
        const bool dist = every && (int64_t)k * cgd.nodes() > kDenseMax &&
                          (double)cgd.nodes() * ratio >= (double)mg->gfine.nodes();
        if (dist) {
          MgLevel C = dist_coarse(ls, *mg, F, cgd, clo, chi);
          mg->lv.push_back(std::move(C));
          ++mg->n_dist;
        }
        else {
          MgLevel C = gathered_coarse(ls, *mg, F);
          mg->lv.push_back(std::move(C));
          break;
        }
      }
    }
    else if (!ls.mg_multi) {
      L.d = Dims{ ls.mg_nx, ls.mg_nx, ls.mg_nz };
      L.nn = L.d.nodes();
      L.n = k * L.nn;
      L.bp = bp;
      L.bc = bc;
      L.v = ls.csr_vals;
      L.dinv = ls.dinv.p;  // computed by ls_solve (k_inv_diag) before the setup
    }
    else {
      // a slab of several ranks: the owned block (ghost columns dropped), padded
      // in z by one decoupled layer when its cell count is odd
      const int pad = ls.mg_nz % 2;
      const Dims own{ ls.mg_nx, ls.mg_nx, ls.mg_nz };
      L.d = Dims{ ls.mg_nx, ls.mg_nx, ls.mg_nz + pad };
      L.nn = L.d.nodes();
      L.n = k * L.nn;
      const int64_t nn_own = own.nodes(), layer = (int64_t)(ls.mg_nx + 1) * (ls.mg_nx + 1);
      DevBuf<int64_t> len;
      len.alloc(L.nn);
      const unsigned g = grid_for(L.nn, 256);
      hipLaunchKernelGGL(k_mg_own_len, dim3(g), dim3(256), 0, ctx.stream, nn_own, L.nn, bp, bc, len.p);
      AFEM_LAUNCHED();
      L.own_bp.alloc(L.nn + 1);
      exclusive_scan_i64(ctx, len.p, L.own_bp.p, L.nn);
      const int64_t nb = read_i64(ctx, L.own_bp.p + L.nn);
      L.own_bc.alloc(nb);
      L.own_v.alloc((size_t)nb * k * k);
      L.own_dinv.alloc(L.n);
      dispatch_k(k, [&](auto kc) {
        constexpr int K = decltype(kc)::value;
        hipLaunchKernelGGL(k_mg_own_copy<K>, dim3(g), dim3(256), 0, ctx.stream, nn_own, L.nn, layer, bp, bc,
                           ls.csr_vals, L.own_bp.p, L.own_bc.p, L.own_v.p);
        AFEM_LAUNCHED();
        hipLaunchKernelGGL(k_mg_dinv<K>, dim3(g), dim3(256), 0, ctx.stream, L.nn, L.own_bp.p, L.own_bc.p, L.own_v.p,
                           L.own_dinv.p);
        AFEM_LAUNCHED();
      });
      ctx.sync();
      L.bp = L.own_bp.p;
      L.bc = L.own_bc.p;
      L.v = L.own_v.p;
      L.dinv = L.own_dinv.p;
    }
    if (!mg->global) mg->lv.push_back(std::move(L));
  }
  while (!mg->lv.back().dist) {
    const MgLevel& F = mg->lv.back();
    if (F.n <= kDenseMax || F.d.nx % 2 || F.d.ny % 2 || F.d.nz % 2 || F.d.nx < 2 || F.d.nz < 2) break;
    MgLevel C;
    C.d = Dims{ F.d.nx / 2, F.d.ny / 2, F.d.nz / 2 };
    C.nn = C.d.nodes();
    C.n = k * C.nn;
    std::vector<int64_t> hbp;
    std::vector<int32_t> hbc;
    coarse_structure(C.d, hbp, hbc);
    C.own_bp.alloc(hbp.size());
    C.own_bc.alloc(hbc.size());
    AFEM_HIP(hipMemcpyAsync(C.own_bp.p, hbp.data(), hbp.size() * 8, hipMemcpyHostToDevice, ctx.stream));
    AFEM_HIP(hipMemcpyAsync(C.own_bc.p, hbc.data(), hbc.size() * 4, hipMemcpyHostToDevice, ctx.stream));
    C.own_v.alloc(hbc.size() * k * k);
    AFEM_HIP(hipMemsetAsync(C.own_v.p, 0, C.own_v.bytes(), ctx.stream));
    C.own_dinv.alloc(C.n);
    const unsigned g = (unsigned)grid_for(C.nn, 128);
    dispatch_k(k, [&](auto kc) {
      constexpr int K = decltype(kc)::value;
      hipLaunchKernelGGL(k_mg_galerkin<K>, dim3(g), dim3(128), 0, ctx.stream, F.d, C.d, F.bp, F.bc, F.v, C.own_bp.p,
                         C.own_bc.p, C.own_v.p, err.p);
      AFEM_LAUNCHED();
      hipLaunchKernelGGL(k_mg_dinv<K>, dim3(g), dim3(128), 0, ctx.stream, C.nn, C.own_bp.p, C.own_bc.p, C.own_v.p,
                         C.own_dinv.p);
      AFEM_LAUNCHED();
    });
    C.bp = C.own_bp.p;
    C.bc = C.own_bc.p;
    C.v = C.own_v.p;
    C.dinv = C.own_dinv.p;
    ctx.sync();  // the host structure vectors go out of scope
    mg->lv.push_back(std::move(C));
  }
  const bool herr = mg->global ? any_rank(ls, err) : [&] {
    int h = 0;
    AFEM_HIP(hipMemcpyAsync(&h, err.p, sizeof(int), hipMemcpyDeviceToHost, ctx.stream));
    ctx.sync();
    return h != 0;
  }();
  AFEM_REQUIRE(!herr, AFEM_ERR_STATE, "multigrid: Galerkin product outside the coarse Kuhn stencil");
  for (size_t l = 0; l < mg->lv.size(); ++l) {
    MgLevel& L = mg->lv[l];
    const bool dist = L.dist;  // vectors with the halo's ghost entries
    L.x.alloc(dist ? L.ncol : L.n);
    L.t.alloc(dist ? L.ncol : L.n);
    L.r.alloc(dist ? L.ncol : L.n);
    if (dist) {
      AFEM_HIP(hipMemsetAsync(L.x.p, 0, L.x.bytes(), ctx.stream));
      AFEM_HIP(hipMemsetAsync(L.t.p, 0, L.t.bytes(), ctx.stream));
      AFEM_HIP(hipMemsetAsync(L.r.p, 0, L.r.bytes(), ctx.stream));
    }
    L.b.alloc(L.n);
    const double lam = dist ? power_lambda_global(ls, *mg, L) : power_lambda(ctx, *mg, L);
    L.omega = lam > 0 ? 4.0 / (3.0 * 1.05 * lam) : 0.6;
    const char* oe = variant("AFEM_MG_OMEGA");  // a factor on every level's omega (measurements)
    if (oe && std::atof(oe) > 0) L.omega *= std::atof(oe);
  }
  MgLevel& Lc = mg->lv.back();
  if (mg->lv.size() > 1 && !Lc.dist && Lc.n <= kDenseMax) dense_inverse(ctx, *mg, Lc);
  // AFEM_MG_KCYCLE=k: levels 1..k of a one-rank hierarchy run the K-cycle
  // (kcycle.hpp) instead of one V-cycle for their coarse problem
  {
    const char* ke = variant("AFEM_MG_KCYCLE");
    const int kcyc = ke ? std::max(0, atoi(ke)) : 0;
    if (!mg->global && mg->partial.n >= 3 * (size_t)kDotGrid)
      for (size_t l = 1; l < mg->lv.size() && (int)l <= kcyc; ++l) {
        MgLevel& L = mg->lv[l];
        if (l + 1 == mg->lv.size() && mg->n_dense == L.n) break;  // solved exactly
        L.kc1.alloc(L.n);
        L.kv1.alloc(L.n);
        L.krt.alloc(L.n);
        L.kcoef.alloc(8);
      }
  }
  mg->key_rows = krows;
  mg->key_vals = ls.csr_vals;
  mg->key_n = ls.n_rows;
  // AFEM_MG_F32 (default 1): block-3 systems' cycle products (smoothing sweeps and residuals,
  // not the PCG's own product) on fp32 copies of the levels' values in k_spmv_blk3f's layout
  // (12 floats per block); the fine copy is refreshed at every solve (its values are
  // re-assembled in place), the coarse operators are fixed with the hierarchy.  =1 the fine
  // level only, =2 (default) every level
  if (k == 3) {
    const char* fe = variant("AFEM_MG_F32");
    const int f32 = fe ? atoi(fe) : 2;
    for (size_t l = 0; l < mg->lv.size() && f32 > 0; ++l) {
      MgLevel& L = mg->lv[l];
      if ((l > 0 && f32 < 2) || L.nn <= 0 || !L.v) continue;
      int64_t nnzb = 0;
      AFEM_HIP(hipMemcpyAsync(&nnzb, L.bp + L.nn, sizeof(int64_t), hipMemcpyDeviceToHost, ctx.stream));
      ctx.sync();
      L.v32.alloc((size_t)(12 * (nnzb > 0 ? nnzb : 1)));
      blk3_to_f32(ctx, L.nn, L.bp, L.v, L.v32.p);
    }
  }
  ls.mg = std::move(mg);
}

namespace {

// `sweeps` damped-Jacobi sweeps on level L from x = 0 (first sweep: omega D^-1 b)
// or from the current iterate; the result is left in L.x
// a product with its epilogue on level L: on the level's fp32 copy when it has one
void level_product(Ctx& ctx, Multigrid& mg, MgLevel& L, int epi, const double* x, double* y, const double* b,
                   const double* dinv, double omega)
{
  if (L.v32.p)
    spmv_blk3f_epi(ctx, epi, L.nn, L.bp, L.bc, L.v32.p, x, y, b, dinv, omega);
  else
    spmv_blk_epi(ctx, mg.k, epi, L.nn, L.bp, L.bc, L.v, x, y, b, dinv, omega);
}

void smooth(Ctx& ctx, Multigrid& mg, MgLevel& L, const double* b, int sweeps, bool from_zero)
{
  const unsigned g = (unsigned)std::min<int64_t>(kVec, (L.n + 255) / 256);
  int s = 0;
  if (from_zero) {
    hipLaunchKernelGGL(k_mg_scale, dim3(g), dim3(256), 0, ctx.stream, L.n, L.omega, L.dinv, b, L.x.p);
    AFEM_LAUNCHED();
    s = 1;
  }
  for (; s < sweeps; ++s) {
    level_product(ctx, mg, L, 1, L.x.p, L.t.p, b, L.dinv, L.omega);
    std::swap(L.x, L.t);
  }
}

void kcycle(Ctx& ctx, Multigrid& mg, size_t l);

// mg_apply's fused entry / exit on level 0 (one rank, block-3 fp32 copy): the first
// sweep already done by k_mg_mask_scale; the last sweep writes z with the
// constraint rows (k_spmv_blk3f<3>) -- done reports it
struct MgExit {
  double* z = nullptr;
  const double* r = nullptr;
  const uint8_t* cons = nullptr;
  const double* dfix = nullptr;
  bool x_ready = false;
  bool done = false;
};

void vcycle(Ctx& ctx, Multigrid& mg, size_t l, const double* b, MgExit* ex = nullptr)
{
  MgLevel& L = mg.lv[l];
  if (l > 0) ex = nullptr;
  if (l + 1 == mg.lv.size()) {
    if (mg.n_dense == L.n && l > 0) {
      hipLaunchKernelGGL(k_mg_gemv, dim3((unsigned)L.n), dim3(64), 0, ctx.stream, (int)L.n, mg.ainv.p, b, L.x.p);
      AFEM_LAUNCHED();
    }
    else {
      smooth(ctx, mg, L, b, l == 0 ? 2 * mg.sweeps : kCoarseSweeps, true);
    }
    return;
  }
  MgLevel& C = mg.lv[l + 1];
  if (ex && ex->x_ready)
    smooth(ctx, mg, L, b, mg.sweeps - 1, false);  // (the first sweep from zero came with the mask)
  else
    smooth(ctx, mg, L, b, mg.sweeps, true);
  level_product(ctx, mg, L, 2, L.x.p, L.r.p, b, nullptr, 0.0);
  dispatch_k(mg.k, [&](auto kc) {
    constexpr int K = decltype(kc)::value;
    hipLaunchKernelGGL(k_mg_restrict<K>, dim3((unsigned)grid_for(C.nn, 256)), dim3(256), 0, ctx.stream, L.d, C.d,
                       L.r.p, C.b.p);
    AFEM_LAUNCHED();
  });
  if (C.kcoef.p)
    kcycle(ctx, mg, l + 1);
  else
    vcycle(ctx, mg, l + 1, C.b.p);
  dispatch_k(mg.k, [&](auto kc) {
    constexpr int K = decltype(kc)::value;
    hipLaunchKernelGGL(k_mg_prolong<K>, dim3((unsigned)grid_for(L.nn, 256)), dim3(256), 0, ctx.stream, L.d, C.d,
                       C.x.p, L.x.p);
    AFEM_LAUNCHED();
  });
  if (ex && L.v32.p && mg.sweeps >= 1) {
    smooth(ctx, mg, L, b, mg.sweeps - 1, false);
    spmv_blk3f_epi(ctx, 3, L.nn, L.bp, L.bc, L.v32.p, L.x.p, ex->z, b, L.dinv, L.omega, ex->cons, ex->r, ex->dfix);
    ex->done = true;
  }
  else {
    smooth(ctx, mg, L, b, mg.sweeps, false);
  }
}

// K-cycle (AFEM_MG_KCYCLE=k, one rank): level l's coarse problem (b in L.b) by
// two flexible-CG steps preconditioned by the cycle at this level (kcycle.hpp)
void kcycle(Ctx& ctx, Multigrid& mg, size_t l)
{
  MgLevel& L = mg.lv[l];
  const int64_t n = L.n;
  const unsigned g = (unsigned)std::min<int64_t>(kVec, (n + 255) / 256);
  const unsigned gd = (unsigned)std::min<int64_t>(kDotGrid, (n + 255) / 256);
  vcycle(ctx, mg, l, L.b.p);
  AFEM_HIP(hipMemcpyAsync(L.kc1.p, L.x.p, n * sizeof(double), hipMemcpyDeviceToDevice, ctx.stream));
  spmv_blk_epi(ctx, mg.k, 0, L.nn, L.bp, L.bc, L.v, L.kc1.p, L.kv1.p, nullptr, nullptr, 0.0);
  hipLaunchKernelGGL(k_kc_dots<2>, dim3(gd), dim3(256), 0, ctx.stream, n, (const double*)L.kc1.p,
                     (const double*)L.kv1.p, (const double*)L.kc1.p, (const double*)L.b.p, (const double*)nullptr,
                     (const double*)nullptr, mg.partial.p);
  hipLaunchKernelGGL(k_kc_coef<1>, dim3(1), dim3(256), 0, ctx.stream, (int)gd, (const double*)mg.partial.p, L.kcoef.p);
  hipLaunchKernelGGL(k_kc_resid, dim3(g), dim3(256), 0, ctx.stream, n, (const double*)L.kcoef.p, (const double*)L.b.p,
                     (const double*)L.kv1.p, L.krt.p);
  AFEM_LAUNCHED();
  vcycle(ctx, mg, l, L.krt.p);
  spmv_blk_epi(ctx, mg.k, 0, L.nn, L.bp, L.bc, L.v, L.x.p, L.t.p, nullptr, nullptr, 0.0);
  hipLaunchKernelGGL(k_kc_dots<3>, dim3(gd), dim3(256), 0, ctx.stream, n, (const double*)L.x.p, (const double*)L.kv1.p,
                     (const double*)L.x.p, (const double*)L.t.p, (const double*)L.x.p, (const double*)L.krt.p,
                     mg.partial.p);
  hipLaunchKernelGGL(k_kc_coef<2>, dim3(1), dim3(256), 0, ctx.stream, (int)gd, (const double*)mg.partial.p, L.kcoef.p);
  hipLaunchKernelGGL(k_kc_comb, dim3(g), dim3(256), 0, ctx.stream, n, (const double*)L.kcoef.p, (const double*)L.kc1.p,
                     L.x.p);
  AFEM_LAUNCHED();
}

// a distributed level of the global V-cycle (the steps of vcycle on the slab's
// owned rows): the level's halo before every product; the restriction to a
// distributed coarse level reads the fine residual's ghost layers, the one to
// the gathered level is summed over the ranks; replicated levels run the same
// arithmetic on every rank
void vcycle_dist(LinearSystem& ls, Multigrid& mg, size_t l, const double* b)
{
  Ctx& ctx = *ls.ctx;
  MgLevel& L = mg.lv[l];
  Halo& H = level_halo(ls, L);
  const bool last = l + 1 == mg.lv.size();
  const int pre = last ? (l == 0 ? 2 * mg.sweeps : kCoarseSweeps) : mg.sweeps;
  smooth(ctx, mg, L, b, 1, true);
  for (int s = 1; s < pre; ++s) {
    halo_exchange(H, ctx, L.x.p);
    smooth(ctx, mg, L, b, 1, false);
  }
  if (last) return;  // coarsest level, distributed: smoothing only (the one-rank counts)
  MgLevel& C = mg.lv[l + 1];
  halo_exchange(H, ctx, L.x.p);
  level_product(ctx, mg, L, 2, L.x.p, L.r.p, b, nullptr, 0.0);
  if (C.dist) {
    halo_exchange(H, ctx, L.r.p);
    dispatch_k(mg.k, [&](auto kc) {
      constexpr int K = decltype(kc)::value;
      hipLaunchKernelGGL(k_mg_restrict_dist<K>, dim3((unsigned)grid_for(C.nn, 256)), dim3(256), 0, ctx.stream, L.gd,
                         L.sm, C.sm, L.r.p, C.b.p);
      AFEM_LAUNCHED();
    });
    vcycle_dist(ls, mg, l + 1, C.b.p);
    halo_exchange(*C.halo, ctx, C.x.p);
    dispatch_k(mg.k, [&](auto kc) {
      constexpr int K = decltype(kc)::value;
      hipLaunchKernelGGL(k_mg_prolong_dist<K>, dim3((unsigned)grid_for(L.nn, 256)), dim3(256), 0, ctx.stream, L.sm,
                         C.sm, C.x.p, L.x.p);
      AFEM_LAUNCHED();
    });
  }
  else {
    dispatch_k(mg.k, [&](auto kc) {
      constexpr int K = decltype(kc)::value;
      hipLaunchKernelGGL(k_mg_restrict_part<K>, dim3((unsigned)grid_for(C.nn, 256)), dim3(256), 0, ctx.stream, L.gd,
                         C.d, L.sm, L.r.p, C.b.p);
      AFEM_LAUNCHED();
    });
    comm_allreduce(ls.halo->comm, ctx, C.b.p, C.n);
    vcycle(ctx, mg, l + 1, C.b.p);
    dispatch_k(mg.k, [&](auto kc) {
      constexpr int K = decltype(kc)::value;
      hipLaunchKernelGGL(k_mg_prolong_own<K>, dim3((unsigned)grid_for(L.nn, 256)), dim3(256), 0, ctx.stream, C.d,
                         L.sm, L.nn, C.x.p, L.x.p);
      AFEM_LAUNCHED();
    });
  }
  for (int s = 0; s < mg.sweeps; ++s) {
    halo_exchange(H, ctx, L.x.p);
    smooth(ctx, mg, L, b, 1, false);
  }
}

}  // namespace

void mg_apply(LinearSystem& ls, const double* r, double* z)
{
  Ctx& ctx = *ls.ctx;
  Multigrid& mg = *ls.mg;
  MgLevel& L0 = mg.lv[0];
  const unsigned g = (unsigned)std::min<int64_t>(kVec, (L0.n + 255) / 256);
  const int64_t n = ls.n_rows;  // < L0.n when the slab's box is padded
  // one rank, block-3 fp32 copy, more than one level: the entry (mask + first sweep) and the
  // exit (last sweep into z + constraint rows) fused (AFEM_MG_FUSE=0: separate passes)
  const char* fe = variant("AFEM_MG_FUSE");
  const bool fuse = !mg.global && n == L0.n && L0.v32.p && mg.lv.size() > 1 && mg.sweeps >= 1 && !(fe && atoi(fe) == 0);
  if (fuse) {
    hipLaunchKernelGGL(k_mg_mask_scale, dim3(g), dim3(256), 0, ctx.stream, L0.n, ls.cons.p, r, L0.omega, L0.dinv,
                       L0.b.p, L0.x.p);
    AFEM_LAUNCHED();
    MgExit ex;
    ex.z = z;
    ex.r = r;
    ex.cons = ls.cons.p;
    ex.dfix = ls.dinv.p;
    ex.x_ready = true;
    vcycle(ctx, mg, 0, L0.b.p, &ex);
    if (ex.done) return;
  }
  else {
    if (n == L0.n)
      hipLaunchKernelGGL(k_mg_mask, dim3(g), dim3(256), 0, ctx.stream, L0.n, ls.cons.p, r, L0.b.p);
    else
      hipLaunchKernelGGL(k_mg_mask_pad, dim3(g), dim3(256), 0, ctx.stream, n, L0.n, ls.cons.p, r, L0.b.p);
    AFEM_LAUNCHED();
    if (mg.global)
      vcycle_dist(ls, mg, 0, L0.b.p);
    else
      vcycle(ctx, mg, 0, L0.b.p);
  }
  AFEM_HIP(hipMemcpyAsync(z, L0.x.p, n * sizeof(double), hipMemcpyDeviceToDevice, ctx.stream));
  hipLaunchKernelGGL(k_mg_fix, dim3(g), dim3(256), 0, ctx.stream, n, ls.cons.p, r, ls.dinv.p, z);
  AFEM_LAUNCHED();
}

}  // namespace afem
