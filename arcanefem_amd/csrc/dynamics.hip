// Device vector kernels of the time-stepping callers of the path
// (modules/elastodynamics/FemModule.cc; modules/passmo/ElastodynamicModule.cc
// reassembles on a fixed structure every step, :469-536).  The per-step
// matrix is re-assembled by afem_bsr_assemble_elasticity_p1_ex (c0 M + K);
// these kernels form the Newmark right-hand side operand and update the
// state.  HBM-bound streaming kernels: 16-B per lane loads, grid-stride.
#include "afem_internal.hpp"

namespace afem {
namespace {

inline unsigned grid_for(int64_t n, int threads)
{
  const int64_t b = (n + threads - 1) / threads;
  return (unsigned)(b < 65535 * 16 ? b : 65535 * 16);
}

// out = a x + b y + c z  (z may be null)
__global__ void k_lincomb(int64_t n, double a, const double* __restrict__ x, double b, const double* __restrict__ y,
                          double c, const double* __restrict__ z, double* __restrict__ out)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double v = a * x[i] + b * y[i];
    if (z) v += c * z[i];
    out[i] = v;
  }
}

// modules/elastodynamics/FemModule.cc:429-455 (_updateVariables):
//   a' = (u_new - u - dt v) / (beta dt^2) - (1 - 2 beta) / (2 beta) a
//   v' = v + dt ((1 - gamma) a + gamma a');  a = a';  u = u_new
__global__ void k_newmark(int64_t n, double dt, double beta, double gamma, const double* __restrict__ un,
                          double* __restrict__ u, double* __restrict__ v, double* __restrict__ a)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double ui = u[i], vi = v[i], ai = a[i], uni = un[i];
    const double an = (uni - ui - dt * vi) / beta / (dt * dt) - (1. - 2. * beta) / 2. / beta * ai;
    v[i] = vi + dt * ((1. - gamma) * ai + gamma * an);
    a[i] = an;
    u[i] = uni;
  }
}

__global__ void k_scatter_vals(int64_t n, const int32_t* __restrict__ ids, const double* __restrict__ vals,
                               double* __restrict__ x)
{
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[ids[i]] = vals[i];
}

}  // namespace

void vec_scatter(Ctx& ctx, int64_t n, const int32_t* ids, const double* vals, double* x)
{
  if (n <= 0) return;
  hipLaunchKernelGGL(k_scatter_vals, dim3(grid_for(n, 256)), dim3(256), 0, ctx.stream, n, ids, vals, x);
  AFEM_LAUNCHED();
}

void vec_lincomb(Ctx& ctx, int64_t n, double a, const double* x, double b, const double* y, double c, const double* z,
                 double* out)
{
  if (n <= 0) return;
  hipLaunchKernelGGL(k_lincomb, dim3(grid_for(n, 256)), dim3(256), 0, ctx.stream, n, a, x, b, y, c, z, out);
  AFEM_LAUNCHED();
}

void newmark_update(Ctx& ctx, int64_t n, double dt, double beta, double gamma, const double* un, double* u, double* v,
                    double* a)
{
  if (n <= 0) return;
  hipLaunchKernelGGL(k_newmark, dim3(grid_for(n, 256)), dim3(256), 0, ctx.stream, n, dt, beta, gamma, un, u, v, a);
  AFEM_LAUNCHED();
}

}  // namespace afem
