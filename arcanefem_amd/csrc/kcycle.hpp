// K-cycle kernels (Notay & Vassilevski's recursive Krylov cycle) shared by the
// algebraic (amg.hip) and geometric (multigrid.hip) hierarchies: a level's
// coarse problem A x = b solved by two flexible-CG steps preconditioned by the
// cycle below, c1 = B b, v1 = A c1, rt = b - alpha1 v1, c2 = B rt, v2 = A c2,
// x = w1 c1 + w2 c2.  The dot products: block partials over a fixed grid,
// summed in a fixed order by one block; every scalar stays on the device.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace afem {
namespace {

constexpr int kDotGrid = 256;
template <int ND>
__global__ __launch_bounds__(256) void k_kc_dots(int64_t n, const double* __restrict__ a0, const double* __restrict__ b0,
                                                  const double* __restrict__ a1, const double* __restrict__ b1,
                                                  const double* __restrict__ a2, const double* __restrict__ b2,
                                                  double* __restrict__ partial)
{
  __shared__ double sh[ND][256];
  double s[3] = { 0.0, 0.0, 0.0 };
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    s[0] += a0[i] * b0[i];
    if (ND > 1) s[1] += a1[i] * b1[i];
    if (ND > 2) s[2] += a2[i] * b2[i];
  }
#pragma unroll
  for (int d = 0; d < ND; ++d) sh[d][threadIdx.x] = s[d];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
#pragma unroll
      for (int d = 0; d < ND; ++d) sh[d][threadIdx.x] += sh[d][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x < ND) partial[ND * blockIdx.x + threadIdx.x] = sh[threadIdx.x][0];
}

// the step coefficients from the partials (one block).  STEP 1: rho1 = c1.v1,
// alpha1 = c1.r / rho1.  STEP 2: gamma = c2.v1, beta = c2.v2, delta = c2.rt,
// alpha2 = delta / (beta - gamma^2 / rho1); x = (alpha1 - gamma alpha2 / rho1) c1
// + alpha2 c2 (coef[2], coef[3]).  A zero or non-positive curvature drops the
// step (its weight 0)
template <int STEP>
__global__ __launch_bounds__(256) void k_kc_coef(int nb, const double* __restrict__ partial, double* __restrict__ coef)
{
  constexpr int ND = STEP == 1 ? 2 : 3;
  __shared__ double sh[ND][256];
  for (int d = 0; d < ND; ++d) sh[d][threadIdx.x] = (int)threadIdx.x < nb ? partial[ND * threadIdx.x + d] : 0.0;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
      for (int d = 0; d < ND; ++d) sh[d][threadIdx.x] += sh[d][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (STEP == 1) {
      const double rho = sh[0][0];
      coef[0] = rho;
      coef[1] = rho > 0.0 ? sh[1][0] / rho : 0.0;
    }
    else {
      const double rho = coef[0], a1 = coef[1];
      const double gam = sh[0][0], bet = sh[1][0], del = sh[2][0];
      const double den = rho > 0.0 ? bet - gam * gam / rho : bet;
      const double a2 = den > 0.0 ? del / den : 0.0;
      coef[2] = rho > 0.0 ? a1 - gam * a2 / rho : a1;
      coef[3] = a2;
    }
  }
}

// several ranks: the partials summed into ND device scalars (one block, fixed
// order), all-reduced by the caller, then the coefficients from the sums
template <int ND>
__global__ __launch_bounds__(256) void k_kc_sum(int nb, const double* __restrict__ partial, double* __restrict__ sums)
{
  __shared__ double sh[ND][256];
  for (int d = 0; d < ND; ++d) sh[d][threadIdx.x] = (int)threadIdx.x < nb ? partial[ND * threadIdx.x + d] : 0.0;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
      for (int d = 0; d < ND; ++d) sh[d][threadIdx.x] += sh[d][threadIdx.x + o];
    __syncthreads();
  }
  if ((int)threadIdx.x < ND) sums[threadIdx.x] = sh[threadIdx.x][0];
}

// k_kc_coef's arithmetic on the (all-reduced) sums
template <int STEP>
__global__ void k_kc_coef_sums(const double* __restrict__ sums, double* __restrict__ coef)
{
  if (threadIdx.x != 0) return;
  if (STEP == 1) {
    const double rho = sums[0];
    coef[0] = rho;
    coef[1] = rho > 0.0 ? sums[1] / rho : 0.0;
  }
  else {
    const double rho = coef[0], a1 = coef[1];
    const double gam = sums[0], bet = sums[1], del = sums[2];
    const double den = rho > 0.0 ? bet - gam * gam / rho : bet;
    const double a2 = den > 0.0 ? del / den : 0.0;
    coef[2] = rho > 0.0 ? a1 - gam * a2 / rho : a1;
    coef[3] = a2;
  }
}

// rt = b - alpha1 v1
__global__ void k_kc_resid(int64_t n, const double* __restrict__ coef, const double* __restrict__ b,
                             const double* __restrict__ v1, double* __restrict__ rt)
{
  const double a1 = coef[1];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    rt[i] = b[i] - a1 * v1[i];
}

// x = w1 c1 + w2 x
__global__ void k_kc_comb(int64_t n, const double* __restrict__ coef, const double* __restrict__ c1,
                            double* __restrict__ x)
{
  const double w1 = coef[2], w2 = coef[3];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] = w1 * c1[i] + w2 * x[i];
}

}  // namespace
}  // namespace afem
