#include <algorithm>
// Device-resident P1 meshes: upload of caller arrays and the synthetic
// jittered structured generator (the benchmark input, DESIGN.md "Synthetic
// inputs").  The generator runs on the GPU so a 1e8-node mesh never crosses
// PCIe; its arithmetic is written with explicitly rounded operations
// (__dmul_rn/__dadd_rn, no FMA contraction) so that the CPU specification in
// oracle/oracle.py::structured_mesh reproduces it bit for bit.
#include "afem_internal.hpp"

namespace afem {
namespace {

__device__ __forceinline__ double hash_u01(uint64_t seed, uint64_t idx)
{
  uint64_t z = seed + (idx + 1ull) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z = z ^ (z >> 31);
  return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

struct Layers {
  int64_t L;         // nodes per layer
  int n_own_layers;  // owned layers k0..k1-1
  int k0, k1;
  int ghost_lo, ghost_hi;
  __device__ __forceinline__ int global_layer(int64_t li) const
  {
    if (li < n_own_layers) return k0 + (int)li;
    if (li == n_own_layers && ghost_lo >= 0) return ghost_lo;
    return ghost_hi;
  }
  __device__ __forceinline__ int local_layer(int k) const
  {
    if (k >= k0 && k < k1) return k - k0;
    if (k == ghost_lo) return n_own_layers;
    return n_own_layers + (ghost_lo >= 0 ? 1 : 0);
  }
};

__global__ void k_gen_coords(int dim, int64_t n_nodes, Layers ly, int np1, double h, double amp, uint64_t seed,
                             double* __restrict__ coords)
{
#pragma clang fp contract(off)  // no a*b+c -> fma here (the file is also built with -ffp-contract=off)
  int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= n_nodes) return;
  int64_t li = l / ly.L, pos = l - li * ly.L;
  int k = ly.global_layer(li);
  int64_t g = pos + (int64_t)k * ly.L;
  int64_t ic[3];
  if (dim == 3) {
    ic[0] = pos % np1;
    ic[1] = pos / np1;
    ic[2] = k;
  }
  else {
    ic[0] = pos;
    ic[1] = k;
    ic[2] = 0;
  }
  for (int c = 0; c < 3; ++c) {
    double x = 0.0;
    if (c < dim) {
      double u = hash_u01(seed, (uint64_t)(g * 3 + c));
      const double a = (double)ic[c] * h;
      const double b = (u - 0.5) * amp;
      x = a + b;
    }
    coords[3 * l + c] = x;
  }
}

// Kuhn subdivision of cube (i,j,k): for each permutation (a0,a1,a2) of the
// axes, the tet (v0, v0+e_a0, v0+e_a0+e_a1, v0+(1,1,1)).
__constant__ int c_kuhn[6][3] = { { 0, 1, 2 }, { 0, 2, 1 }, { 1, 0, 2 }, { 1, 2, 0 }, { 2, 0, 1 }, { 2, 1, 0 } };

__global__ void k_gen_tets(int64_t n_cells, int n, int c_lo, Layers ly, int32_t* __restrict__ cn)
{
  int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_cells) return;
  int64_t cube = c / 6;
  int t = (int)(c - cube * 6);
  int ci = (int)(cube % n);
  int cj = (int)((cube / n) % n);
  int ck = c_lo + (int)(cube / ((int64_t)n * n));
  int v[3] = { ci, cj, ck };
  int np1 = n + 1;
  auto lid = [&](int i, int j, int k) -> int32_t {
    return (int32_t)((int64_t)ly.local_layer(k) * ly.L + i + (int64_t)np1 * j);
  };
  cn[4 * c + 0] = lid(v[0], v[1], v[2]);
  v[c_kuhn[t][0]] += 1;
  cn[4 * c + 1] = lid(v[0], v[1], v[2]);
  v[c_kuhn[t][1]] += 1;
  cn[4 * c + 2] = lid(v[0], v[1], v[2]);
  cn[4 * c + 3] = lid(ci + 1, cj + 1, ck + 1);
}

__global__ void k_gen_tris(int64_t n_cells, int n, int c_lo, Layers ly, int32_t* __restrict__ cn)
{
  int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_cells) return;
  int64_t sq = c / 2;
  int t = (int)(c - sq * 2);
  int i = (int)(sq % n);
  int j = c_lo + (int)(sq / n);
  auto lid = [&](int ii, int jj) -> int32_t { return (int32_t)((int64_t)ly.local_layer(jj) * ly.L + ii); };
  int32_t v00 = lid(i, j), v10 = lid(i + 1, j), v11 = lid(i + 1, j + 1), v01 = lid(i, j + 1);
  if (t == 0) {
    cn[3 * c + 0] = v00;
    cn[3 * c + 1] = v10;
    cn[3 * c + 2] = v11;
  }
  else {
    cn[3 * c + 0] = v00;
    cn[3 * c + 1] = v11;
    cn[3 * c + 2] = v01;
  }
}

__global__ void k_local_to_global(int64_t n_nodes, Layers ly, int64_t* __restrict__ out)
{
  int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= n_nodes) return;
  int64_t li = l / ly.L, pos = l - li * ly.L;
  out[l] = pos + (int64_t)ly.global_layer(li) * ly.L;
}

Layers layers_of(const StructuredInfo& st)
{
  Layers ly;
  ly.L = st.L;
  ly.k0 = st.k0;
  ly.k1 = st.k1;
  ly.n_own_layers = st.k1 - st.k0;
  ly.ghost_lo = st.ghost_lo;
  ly.ghost_hi = st.ghost_hi;
  return ly;
}

inline unsigned grid_for(int64_t n, int threads) { return (unsigned)((n + threads - 1) / threads); }

}  // namespace

void mesh_structured(Ctx& ctx, Mesh& m, int dim, int n, int nz, double jitter, uint64_t seed, int nranks, int rank)
{
  AFEM_REQUIRE(dim == 2 || dim == 3, AFEM_ERR_ARG, "structured mesh: dim must be 2 or 3");
  AFEM_REQUIRE(n >= 1, AFEM_ERR_ARG, "structured mesh: n must be >= 1");
  if (dim == 2 || nz <= 0) nz = n;
  AFEM_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, AFEM_ERR_ARG, "structured mesh: bad rank/nranks");
  StructuredInfo& st = m.st;
  st.valid = true;
  st.dim = dim;
  st.n = n;
  st.nz = nz;
  st.nranks = nranks;
  st.rank = rank;
  st.jitter = jitter;
  st.seed = seed;
  st.L = (dim == 3) ? (int64_t)(n + 1) * (n + 1) : (int64_t)(n + 1);
  const int nlayers = nz + 1;
  AFEM_REQUIRE(nranks <= nlayers, AFEM_ERR_ARG, "structured mesh: more ranks than node layers");
  st.k0 = (int)((int64_t)rank * nlayers / nranks);
  st.k1 = (int)((int64_t)(rank + 1) * nlayers / nranks);
  st.ghost_lo = st.k0 > 0 ? st.k0 - 1 : -1;
  st.ghost_hi = st.k1 < nlayers ? st.k1 : -1;
  const int nl_local = (st.k1 - st.k0) + (st.ghost_lo >= 0) + (st.ghost_hi >= 0);
  m.ctx = &ctx;
  m.dim = dim;
  m.nv = dim + 1;
  m.n_nodes = (int64_t)nl_local * st.L;
  m.n_own = (int64_t)(st.k1 - st.k0) * st.L;
  AFEM_REQUIRE(m.n_nodes < (int64_t)INT32_MAX, AFEM_ERR_LIMIT, "structured mesh: more than 2^31-1 local nodes");
  const int c_lo = st.k0 > 0 ? st.k0 - 1 : 0;
  const int c_hi = st.k1 < nz ? st.k1 : nz;
  const int64_t per_layer = (dim == 3) ? (int64_t)n * n * 6 : (int64_t)n * 2;
  m.n_cells = (int64_t)(c_hi - c_lo) * per_layer;
  m.coords.alloc((size_t)m.n_nodes * 3);
  m.cell_node.alloc((size_t)m.n_cells * m.nv);
  Layers ly = layers_of(st);
  const double h = 1.0 / n;
  const double amp = jitter * h;
  ctx.set_device();
  if (m.n_nodes) {
    hipLaunchKernelGGL(k_gen_coords, dim3(grid_for(m.n_nodes, 256)), dim3(256), 0, ctx.stream, dim, m.n_nodes, ly,
                       n + 1, h, amp, seed, m.coords.p);
    AFEM_LAUNCHED();
  }
  if (m.n_cells) {
    if (dim == 3)
      hipLaunchKernelGGL(k_gen_tets, dim3(grid_for(m.n_cells, 256)), dim3(256), 0, ctx.stream, m.n_cells, n, c_lo, ly,
                         m.cell_node.p);
    else
      hipLaunchKernelGGL(k_gen_tris, dim3(grid_for(m.n_cells, 256)), dim3(256), 0, ctx.stream, m.n_cells, n, c_lo, ly,
                         m.cell_node.p);
    AFEM_LAUNCHED();
  }
}

void mesh_local_to_global(Mesh& m, int64_t* host_out)
{
  Ctx& ctx = *m.ctx;
  if (m.part.valid) {
    std::copy(m.part.l2g.begin(), m.part.l2g.end(), host_out);
    return;
  }
  if (!m.st.valid) {
    for (int64_t i = 0; i < m.n_nodes; ++i) host_out[i] = i;
    return;
  }
  DevBuf<int64_t> d;
  d.alloc(m.n_nodes);
  hipLaunchKernelGGL(k_local_to_global, dim3(grid_for(m.n_nodes, 256)), dim3(256), 0, ctx.stream, m.n_nodes,
                     layers_of(m.st), d.p);
  AFEM_LAUNCHED();
  AFEM_HIP(hipMemcpyAsync(host_out, d.p, d.bytes(), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
}

void mesh_structured_bottom(Mesh& m, std::vector<int32_t>& ids)
{
  ids.clear();
  AFEM_REQUIRE(m.st.valid, AFEM_ERR_ARG, "mesh is not structured");
  if (m.st.k0 != 0) return;
  ids.resize(m.st.L);
  for (int64_t i = 0; i < m.st.L; ++i) ids[i] = (int32_t)i;
}

}  // namespace afem
