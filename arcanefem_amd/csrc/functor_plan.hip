// Cell-unit plan of a structure for generic element functors (one-time,
// device): what the atomic-free cell kernel of
// include/arcanefem_amd_generic.hpp (afem::generic::assemble_bilinear, the
// module's own element lambda, femutils/BSRFormat.h:1105-1111) walks.
//
// The reference's BSRFormat::assembleBilinearAtomic (femutils/BSRFormat.h:
// 786-837) evaluates the functor once per cell and adds 16 k^2 f64 atomics
// into global memory after a linear column search; its atomic-free variant
// (:937-1100) evaluates it once per (row, cell), 4x the element arithmetic.
// Here a wavefront owns a UNIT of rows whose blocks stay in LDS: the cells
// incident to the unit are evaluated once per unit, the unit's own rows are
// accumulated in LDS, every value is written to HBM once.  The redundant
// evaluations (cells shared by two units) are what the unit shape bounds:
//
//  * lattice meshes (the generator's boxes, array-fed meshes whose owned
//    nodes sit on a lattice): a unit is a column of fx x fy nodes over zs
//    consecutive z layers, processed layer by layer (every cell spans at most
//    two consecutive layers, checked), so only two layers of rows are live in
//    LDS and the column's cells are shared with its neighbour columns only:
//    1 + 1/fx + 1/fy + 1/zs evaluations per cell (C2's default 8 x 8 x 10:
//    1.34, against 1.75 for the 4x4x4 bricks of the strip kernels; zs from a
//    target of 16384 units: 3 % faster than 8192 units of zs 20, r04e);
//  * other meshes: rl-row pieces of the structure's processing-order slices
//    (Hilbert-ordered), one layer.
//
// A unit's cells come in stages (stage L = the cells whose highest in-unit
// vertex lies in layer L), each cell once per unit, sorted by a key built from
// the in-unit vertex pattern and lane positions: the chunks of 64 cells a wave
// evaluates together are mostly translates of one cell type, so their LDS
// additions hit distinct rows.  Each entry carries the row position (layer
// parity, lane) of every in-unit vertex and the slot of every vertex in that
// row, found once here by a binary search of the sorted row.
#include "afem_internal.hpp"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace afem {
namespace {

inline unsigned grid_for(int64_t n, int threads) { return (unsigned)((n + threads - 1) / threads); }

struct UnitGeom {
  int lattice;              // 1: lattice columns with z layers; 0: slice pieces (one layer)
  int64_t Lx, Ly, Lz;       // lattice layer counts
  int fx, fy, zs, rl;       // footprint, layers per segment, lanes per layer
  int64_t tx, ty, ns;       // columns along x / y, segments along z
  int nv;
  int64_t n_own;
};

__host__ __device__ inline int64_t unit_first_stage(const UnitGeom& g, int64_t u)
{
  if (!g.lattice) return u;
  const int64_t col = u / g.ns, seg = u - col * g.ns;
  return col * g.Lz + seg * g.zs;
}
__host__ __device__ inline int unit_layers(const UnitGeom& g, int64_t u)
{
  if (!g.lattice) return 1;
  const int64_t seg = u % g.ns;
  const int64_t rest = g.Lz - seg * g.zs;
  return (int)(rest < g.zs ? rest : g.zs);
}
__device__ inline int64_t stage_unit(const UnitGeom& g, int64_t si)
{
  if (!g.lattice) return si;
  const int64_t col = si / g.Lz, z = si - col * g.Lz;
  return col * g.ns + z / g.zs;
}

// generator boxes: owned node l = x + (n+1) (y + (n+1) z) (mesh.hip k_gen_coords)
__global__ void k_gen_lattice(int64_t n_rows, int64_t ax, int64_t ay, int32_t* __restrict__ lx,
                              int32_t* __restrict__ ly, int32_t* __restrict__ lz)
{
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rows) return;
  const int64_t L = ax * ay, z = r / L, p = r - z * L;
  lx[r] = (int32_t)(p % ax);
  ly[r] = (int32_t)(p / ax);
  lz[r] = (int32_t)z;
}

// row -> (unit, layer << 8 | lane), and the unit's layer rows
__global__ void k_rowmap_lattice(int64_t n_rows, const int32_t* __restrict__ lx, const int32_t* __restrict__ ly,
                                 const int32_t* __restrict__ lz, UnitGeom g, int32_t* __restrict__ r_unit,
                                 int32_t* __restrict__ r_li, int32_t* __restrict__ lrows)
{
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rows) return;
  const int64_t x = lx[r], y = ly[r], z = lz[r];
  const int64_t u = ((y / g.fy) * g.tx + x / g.fx) * g.ns + z / g.zs;
  const int layer = (int)(z % g.zs);
  const int lane = (int)((y % g.fy) * g.fx + x % g.fx);
  r_unit[r] = (int32_t)u;
  r_li[r] = layer << 8 | lane;
  lrows[(unit_first_stage(g, u) + layer) * g.rl + lane] = (int32_t)r;
}

__global__ void k_rowmap_slices(int64_t n_pos, const int32_t* __restrict__ perm, int rl, int32_t* __restrict__ r_unit,
                                int32_t* __restrict__ r_li, int32_t* __restrict__ lrows)
{
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pos) return;
  const int32_t r = perm[p];
  if (r < 0) return;
  r_unit[r] = (int32_t)(p / rl);
  r_li[r] = (int32_t)(p % rl);
  lrows[p] = r;
}

// The cells node r claims: those incident to r's unit whose highest in-unit
// vertex layer is r's layer and whose first vertex (cell order) in that layer
// is r.  WRITE = false counts them (and flags a cell spanning more than two
// layers), true emits (stage index << 32 | order key, cell).
template <int NV, bool WRITE>
__global__ void k_claims(int64_t n_rows, const int32_t* __restrict__ cn, const int64_t* __restrict__ nc_ptr,
                         const int32_t* __restrict__ nc, const int32_t* __restrict__ r_unit,
                         const int32_t* __restrict__ r_li, UnitGeom g, int32_t* __restrict__ cnt,
                         const int64_t* __restrict__ off, unsigned long long* __restrict__ keys,
                         int32_t* __restrict__ vals, int32_t* __restrict__ err)
{
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rows) return;
  const int32_t u = r_unit[r];
  const int64_t first = unit_first_stage(g, u);
  int n = 0;
  int64_t o = WRITE ? off[r] : 0;
  for (int64_t k = nc_ptr[r]; k < nc_ptr[r + 1]; ++k) {
    const int32_t c = nc[k];
    int32_t v[NV], lay[NV], lane[NV];
    bool in[NV];
    int top = -1, bot = 1 << 30;
#pragma unroll
    for (int a = 0; a < NV; ++a) {
      v[a] = cn[(int64_t)c * NV + a];
      in[a] = v[a] >= 0 && v[a] < g.n_own && r_unit[v[a]] == u;
      const int li = in[a] ? r_li[v[a]] : 0;
      lay[a] = in[a] ? li >> 8 : -1;
      lane[a] = in[a] ? li & 0xff : 63;
      if (in[a]) {
        top = lay[a] > top ? lay[a] : top;
        bot = lay[a] < bot ? lay[a] : bot;
      }
    }
    if (top - bot > 1) {
      if (!WRITE) atomicOr(err, 1);
      continue;
    }
    int claimer = -1;
#pragma unroll
    for (int a = NV - 1; a >= 0; --a)
      if (in[a] && lay[a] == top) claimer = a;
    if (claimer < 0 || v[claimer] != (int32_t)r) continue;
    if (WRITE) {
      uint32_t pat = 0, lanes = 0;
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const bool ia = a < NV && in[a];
        pat |= (uint32_t)((ia ? 2 : 0) | (ia && lay[a] == top ? 1 : 0)) << (2 * (3 - a));
        lanes |= (uint32_t)(ia ? lane[a] & 63 : 63) << (6 * (3 - a));
      }
      keys[o] = (unsigned long long)(first + top) << 32 | (unsigned long long)(pat << 24 | lanes);
      vals[o] = c;
      ++o;
    }
    ++n;
  }
  if (!WRITE) cnt[r] = n;
}

// stage_ptr[s] = first sorted entry of stage s (entries sorted by stage index)
__global__ void k_stage_ptr(int64_t n_ent, const unsigned long long* __restrict__ keys, int64_t n_stages,
                            int64_t* __restrict__ stage_ptr)
{
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_ent) return;
  const int64_t si = (int64_t)(keys[e] >> 32);
  const int64_t prev = e > 0 ? (int64_t)(keys[e - 1] >> 32) : -1;
  for (int64_t s = prev + 1; s <= si; ++s) stage_ptr[s] = e;
  if (e == n_ent - 1)
    for (int64_t s = si + 1; s <= n_stages; ++s) stage_ptr[s] = n_ent;
}

__device__ int slot_of(const int32_t* __restrict__ c, int len, int32_t x)
{
  int lo = 0, hi = len;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (c[mid] < x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo < len && c[lo] == x ? lo : -1;
}

template <int NV, bool WIDE>
__global__ void k_fill_entries(int64_t n_ent, const unsigned long long* __restrict__ keys,
                               const int32_t* __restrict__ vals, UnitGeom g, const int32_t* __restrict__ cn,
                               const int32_t* __restrict__ r_unit, const int32_t* __restrict__ r_li,
                               const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ cols,
                               uint32_t* __restrict__ ent, uint32_t* __restrict__ ent2, int32_t* __restrict__ err)
{
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_ent) return;
  const int64_t u = stage_unit(g, (int64_t)(keys[e] >> 32));
  const int32_t c = vals[e];
  int32_t v[NV];
#pragma unroll
  for (int a = 0; a < NV; ++a) v[a] = cn[(int64_t)c * NV + a];
  uint32_t pos = 0, sl[4] = { 0, 0, 0, 0 };
#pragma unroll
  for (int a = 0; a < NV; ++a) {
    if (v[a] < 0 || v[a] >= g.n_own || r_unit[v[a]] != u) continue;
    const int li = r_li[v[a]];
    pos |= (0x80u | (uint32_t)((li >> 8) & 1) << 6 | (uint32_t)(li & 63)) << (8 * a);
    const int32_t* rc = cols + row_ptr[v[a]];
    const int len = (int)(row_ptr[v[a] + 1] - row_ptr[v[a]]);
#pragma unroll
    for (int b = 0; b < NV; ++b) {
      const int s = slot_of(rc, len, v[b]);
      if (s < 0 || (!WIDE && s > 15) || s > 255) {
        atomicOr(err, 2);
        continue;
      }
      sl[a] |= (uint32_t)s << ((WIDE ? 8 : 4) * b);
    }
  }
  if (WIDE) {
    reinterpret_cast<uint4*>(ent)[e] = make_uint4(sl[0], sl[1], sl[2], sl[3]);
    reinterpret_cast<uint2*>(ent2)[e] = make_uint2((uint32_t)c, pos);
  }
  else {
    reinterpret_cast<uint4*>(ent)[e] = make_uint4((uint32_t)c, sl[0] | sl[1] << 16, sl[2] | sl[3] << 16, pos);
  }
}

// packed entries: the distinct (slots 0|1, slots 2|3, positions) words of the
// compact entries, numbered in the order (positions with vertex 0's byte
// first, then slots: two stable radix passes, slots first) -- the order of
// the stage sort's lane key, so that the 64 translates of one cell a wave
// evaluates together read consecutive patterns (a few cache lines, not 64);
// an entry keeps its cell and the number
__global__ void k_pat_key_slots(int64_t n, const uint32_t* __restrict__ ent, unsigned long long* __restrict__ key,
                                int32_t* __restrict__ idx)
{
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  key[e] = (unsigned long long)ent[4 * e + 1] | (unsigned long long)ent[4 * e + 2] << 32;
  idx[e] = (int32_t)e;
}

__global__ void k_pat_key_pos(int64_t n, const uint32_t* __restrict__ ent, const int32_t* __restrict__ idx,
                              uint32_t* __restrict__ key)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  key[i] = __builtin_bswap32(ent[4 * (int64_t)idx[i] + 3]);
}

__global__ void k_pat_flags(int64_t n, const uint32_t* __restrict__ ent, const int32_t* __restrict__ idx,
                            int32_t* __restrict__ flag)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int f = 1;
  if (i > 0) {
    const int64_t a = idx[i], b = idx[i - 1];
    f = ent[4 * a + 1] != ent[4 * b + 1] || ent[4 * a + 2] != ent[4 * b + 2] || ent[4 * a + 3] != ent[4 * b + 3];
  }
  flag[i] = f;
}

__global__ void k_pat_emit(int64_t n, const uint32_t* __restrict__ ent, const int32_t* __restrict__ idx,
                           const int32_t* __restrict__ flag, const int32_t* __restrict__ pid,
                           uint32_t* __restrict__ patterns, uint32_t* __restrict__ packed)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t e = idx[i];
  const int32_t q = pid[i] - 1;
  const uint4 w = reinterpret_cast<const uint4*>(ent)[e];
  if (flag[i]) reinterpret_cast<uint4*>(patterns)[q] = make_uint4(0u, w.y, w.z, w.w);
  reinterpret_cast<uint2*>(packed)[e] = make_uint2(w.x, (uint32_t)q);
}

// Replaces the compact entries by packed ones (AFEM_FUNCTOR_PACKED=1: always;
// =auto: when the table, 16 B per pattern, is at most half of the 8 B per
// entry saved and within 4 MB, one XCD's L2).  Off by default: C2 has 2901
// patterns and 0.64 GB less traffic per launch, but the pattern gather -- one
// more 64-lane, 64-line load per evaluation group, prefetched a group ahead --
// costs more than the bytes save (r05o, one process: module element 1.83 vs
// 1.77 ms, lean element 1.47 vs 1.30 ms).
void pack_entries(Ctx& ctx, FunctorPlan& P)
{
  const int64_t n = P.n_entries;
  const char* pe = variant("AFEM_FUNCTOR_PACKED");
  if (P.wide || n <= 0 || !pe || (std::string(pe) != "1" && std::string(pe) != "auto")) return;
  DevBuf<unsigned long long> k64, k64s;
  DevBuf<int32_t> idx, idx1;
  k64.alloc(n);
  k64s.alloc(n);
  idx.alloc(n);
  idx1.alloc(n);
  hipLaunchKernelGGL(k_pat_key_slots, dim3(grid_for(n, 256)), dim3(256), 0, ctx.stream, n, P.ent.p, k64.p, idx.p);
  AFEM_LAUNCHED();
  size_t tb = 0;
  AFEM_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k64.p, k64s.p, idx.p, idx1.p, (int)n, 0, 64, ctx.stream));
  DevBuf<unsigned char> tmp;
  tmp.alloc(tb > 0 ? tb : 1);
  AFEM_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, k64.p, k64s.p, idx.p, idx1.p, (int)n, 0, 64, ctx.stream));
  k64.reset();
  k64s.reset();
  DevBuf<uint32_t> k32, k32s;
  k32.alloc(n);
  k32s.alloc(n);
  hipLaunchKernelGGL(k_pat_key_pos, dim3(grid_for(n, 256)), dim3(256), 0, ctx.stream, n, P.ent.p, idx1.p, k32.p);
  AFEM_LAUNCHED();
  size_t tb2 = 0;
  AFEM_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb2, k32.p, k32s.p, idx1.p, idx.p, (int)n, 0, 32, ctx.stream));
  if (tb2 > tb) tmp.alloc(tb2);
  AFEM_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb2, k32.p, k32s.p, idx1.p, idx.p, (int)n, 0, 32, ctx.stream));
  k32.reset();
  k32s.reset();
  // idx: entries in (positions, slots) order
  DevBuf<int32_t>& flag = idx1;
  hipLaunchKernelGGL(k_pat_flags, dim3(grid_for(n, 256)), dim3(256), 0, ctx.stream, n, P.ent.p, idx.p, flag.p);
  AFEM_LAUNCHED();
  DevBuf<int32_t> pid;
  pid.alloc(n);
  size_t tb3 = 0;
  AFEM_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tb3, flag.p, pid.p, (int)n, ctx.stream));
  if (tb3 > tmp.bytes()) tmp.alloc(tb3);
  AFEM_HIP(hipcub::DeviceScan::InclusiveSum(tmp.p, tb3, flag.p, pid.p, (int)n, ctx.stream));
  int32_t n_pat = 0;
  AFEM_HIP(hipMemcpyAsync(&n_pat, pid.p + (n - 1), sizeof(n_pat), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  P.n_patterns = n_pat;
  const bool force = pe && std::string(pe) == "1";
  if (!force && ((int64_t)n_pat > n / 4 || (int64_t)n_pat * 16 > (4 << 20))) return;
  P.patterns.alloc((size_t)n_pat * 4);
  DevBuf<uint32_t> packed;
  packed.alloc((size_t)n * 2);
  hipLaunchKernelGGL(k_pat_emit, dim3(grid_for(n, 256)), dim3(256), 0, ctx.stream, n, P.ent.p, idx.p, flag.p, pid.p,
                     P.patterns.p, packed.p);
  AFEM_LAUNCHED();
  ctx.sync();
  std::swap(P.ent, packed);
  P.packed = 1;
}

// unit records; flag 1 when every layer's lanes 8q..8q+7 hold a prefix of
// consecutive rows (their values are one contiguous range: coalesced stores)
__global__ void k_units(int64_t n_units, UnitGeom g, const int32_t* __restrict__ lrows, int runs_ok,
                        afem_functor_unit* __restrict__ units)
{
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= n_units) return;
  afem_functor_unit U;
  U.first_stage = unit_first_stage(g, u);
  U.n_stages = unit_layers(g, u);
  int ok = runs_ok;
  for (int L = 0; L < U.n_stages && ok; ++L) {
    const int32_t* lr = lrows + (U.first_stage + L) * g.rl;
    for (int q = 0; q < g.rl / 8 && ok; ++q) {
      bool ended = false;
      for (int i = 0; i < 8; ++i) {
        const int32_t r = lr[8 * q + i];
        if (r < 0) {
          ended = true;
          continue;
        }
        if (ended || (i > 0 && r != lr[8 * q + i - 1] + 1)) ok = 0;
      }
    }
  }
  U.flags = ok;
  units[u] = U;
}

__global__ void k_count_flags(int64_t n, const afem_functor_unit* __restrict__ units, unsigned long long* out)
{
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u < n && (units[u].flags & 1)) atomicAdd(out, 1ull);
}

// Unit rows of a non-lattice plan grown as clusters (round 6): in the
// processing (Hilbert) order, every row not yet taken seeds a unit that takes
// rows breadth first over the structure's couplings until it holds rl rows;
// the unit's LDS rows are then a compact blob of the mesh instead of rl
// consecutive curve positions, and fewer of its cells are shared with other
// units (L-shape-3D refined 5x, emulated: 2.02 -> 1.80 evaluations per cell
// against 64-node Morton pieces).  Out: the position -> row map (rl per unit,
// -1 = idle lane) and the unit count.  AFEM_FUNCTOR_CLUSTER=0: the curve
// pieces (k_rowmap_slices).
std::vector<int32_t> cluster_positions(Ctx& ctx, const Structure& s, int rl, int64_t& n_units)
{
  const int64_t n = s.n_rows;
  std::vector<int64_t> rp(n + 1);
  std::vector<int32_t> perm((size_t)s.n_slices * 64);
  AFEM_HIP(hipMemcpyAsync(rp.data(), s.row_ptr.p, (n + 1) * 8, hipMemcpyDeviceToHost, ctx.stream));
  AFEM_HIP(hipMemcpyAsync(perm.data(), s.perm.p, perm.size() * 4, hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  std::vector<int32_t> ci(rp[n]);
  if (rp[n]) AFEM_HIP(hipMemcpyAsync(ci.data(), s.cols.p, rp[n] * 4, hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  std::vector<int32_t> unit_of(n, -1);
  std::vector<int32_t> pos;
  pos.reserve((size_t)n + n / 8);
  std::vector<int32_t> q;
  q.reserve(rl);
  int64_t u = 0;
  for (int32_t seed : perm) {
    if (seed < 0 || seed >= n || unit_of[seed] >= 0) continue;
    q.clear();
    q.push_back(seed);
    unit_of[seed] = (int32_t)u;
    for (size_t h = 0; h < q.size() && (int)q.size() < rl; ++h) {
      const int32_t v = q[h];
      for (int64_t k = rp[v]; k < rp[v + 1] && (int)q.size() < rl; ++k) {
        const int32_t w = ci[k];
        if (w < 0 || w >= n || unit_of[w] >= 0) continue;
        unit_of[w] = (int32_t)u;
        q.push_back(w);
      }
    }
    for (int t = 0; t < rl; ++t) pos.push_back(t < (int)q.size() ? q[t] : -1);
    ++u;
  }
  n_units = u;
  return pos;
}

__global__ void k_rowmap_positions(int64_t n_pos, const int32_t* __restrict__ pos, int rl, int32_t* __restrict__ r_unit,
                                   int32_t* __restrict__ r_li, int32_t* __restrict__ lrows)
{
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pos) return;
  const int32_t r = pos[p];
  lrows[p] = r;
  if (r < 0) return;
  r_unit[r] = (int32_t)(p / rl);
  r_li[r] = (int32_t)(p % rl);
}

int64_t env_int(const char* name, int64_t dflt)
{
  const char* v = variant(name);
  return v && *v ? std::atoll(v) : dflt;
}

template <int NV>
void build_entries(Ctx& ctx, Bsr& b, const UnitGeom& g, const DevBuf<int64_t>& nc_ptr, const DevBuf<int32_t>& nc,
                   const DevBuf<int32_t>& r_unit, const DevBuf<int32_t>& r_li, DevBuf<int32_t>& err, bool& span_ok)
{
  Mesh& m = *b.mesh;
  Structure& s = b.s;
  FunctorPlan& P = b.fplan;
  const int64_t n_rows = s.n_rows;
  DevBuf<int32_t> cnt;
  DevBuf<int64_t> off;
  cnt.alloc(n_rows);
  off.alloc(n_rows + 1);
  AFEM_HIP(hipMemsetAsync(err.p, 0, err.bytes(), ctx.stream));
  hipLaunchKernelGGL((k_claims<NV, false>), dim3(grid_for(n_rows, 256)), dim3(256), 0, ctx.stream, n_rows,
                     m.cell_node.p, nc_ptr.p, nc.p, r_unit.p, r_li.p, g, cnt.p, nullptr, nullptr, nullptr, err.p);
  AFEM_LAUNCHED();
  int32_t herr = 0;
  AFEM_HIP(hipMemcpyAsync(&herr, err.p, sizeof(herr), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  span_ok = herr == 0;
  if (!span_ok) return;
  exclusive_scan_i32_to_i64(ctx, cnt.p, off.p, n_rows);
  const int64_t n_ent = read_i64(ctx, off.p + n_rows);
  AFEM_REQUIRE(n_ent < (int64_t)INT32_MAX, AFEM_ERR_LIMIT, "functor plan: more than 2^31 cell evaluations");
  DevBuf<unsigned long long> keys, keys_s;
  DevBuf<int32_t> vals, vals_s;
  keys.alloc(n_ent > 0 ? n_ent : 1);
  keys_s.alloc(n_ent > 0 ? n_ent : 1);
  vals.alloc(n_ent > 0 ? n_ent : 1);
  vals_s.alloc(n_ent > 0 ? n_ent : 1);
  hipLaunchKernelGGL((k_claims<NV, true>), dim3(grid_for(n_rows, 256)), dim3(256), 0, ctx.stream, n_rows,
                     m.cell_node.p, nc_ptr.p, nc.p, r_unit.p, r_li.p, g, cnt.p, off.p, keys.p, vals.p, err.p);
  AFEM_LAUNCHED();
  cnt.reset();
  off.reset();
  if (n_ent > 0) {
    int end_bit = 32;
    while (end_bit < 64 && (P.n_stages >> (end_bit - 32)) > 0) ++end_bit;
    size_t tmp_bytes = 0;
    AFEM_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, keys.p, keys_s.p, vals.p, vals_s.p, (int)n_ent, 0,
                                                end_bit, ctx.stream));
    DevBuf<unsigned char> tmp;
    tmp.alloc(tmp_bytes > 0 ? tmp_bytes : 1);
    AFEM_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.p, tmp_bytes, keys.p, keys_s.p, vals.p, vals_s.p, (int)n_ent, 0,
                                                end_bit, ctx.stream));
  }
  keys.reset();
  vals.reset();
  P.n_entries = n_ent;
  P.stage_ptr.alloc(P.n_stages + 1);
  AFEM_HIP(hipMemsetAsync(P.stage_ptr.p, 0, P.stage_ptr.bytes(), ctx.stream));
  if (n_ent > 0) {
    hipLaunchKernelGGL(k_stage_ptr, dim3(grid_for(n_ent, 256)), dim3(256), 0, ctx.stream, n_ent, keys_s.p, P.n_stages,
                       P.stage_ptr.p);
    AFEM_LAUNCHED();
  }
  P.ent.alloc((size_t)(n_ent > 0 ? n_ent : 1) * 4);
  if (P.wide) P.ent2.alloc((size_t)(n_ent > 0 ? n_ent : 1) * 2);
  if (n_ent > 0) {
    if (P.wide)
      hipLaunchKernelGGL((k_fill_entries<NV, true>), dim3(grid_for(n_ent, 256)), dim3(256), 0, ctx.stream, n_ent,
                         keys_s.p, vals_s.p, g, m.cell_node.p, r_unit.p, r_li.p, s.row_ptr.p, s.cols.p, P.ent.p,
                         P.ent2.p, err.p);
    else
      hipLaunchKernelGGL((k_fill_entries<NV, false>), dim3(grid_for(n_ent, 256)), dim3(256), 0, ctx.stream, n_ent,
                         keys_s.p, vals_s.p, g, m.cell_node.p, r_unit.p, r_li.p, s.row_ptr.p, s.cols.p, P.ent.p,
                         nullptr, err.p);
    AFEM_LAUNCHED();
  }
  AFEM_HIP(hipMemcpyAsync(&herr, err.p, sizeof(herr), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  AFEM_REQUIRE(herr == 0, AFEM_ERR_STATE, "functor plan: a cell couples nodes outside the sparsity");
  pack_entries(ctx, P);
}

}  // namespace

void functor_plan_build(Bsr& b)
{
  Mesh& m = *b.mesh;
  Ctx& ctx = *m.ctx;
  Structure& s = b.s;
  FunctorPlan& P = b.fplan;
  P = FunctorPlan();
  const int k = b.nb_dof;
  AFEM_REQUIRE(k >= 1 && k <= 3, AFEM_ERR_NOT_IMPL, "functor plan: NB_DOF 1..3");
  AFEM_REQUIRE(m.nv == 3 || m.nv == 4, AFEM_ERR_NOT_IMPL, "functor plan: P1 triangles or tetrahedra");
  const int64_t n_rows = s.n_rows;
  P.nb_dof = k;
  P.w = s.max_row_len;
  P.wide = P.w > 16 ? 1 : 0;

  DevBuf<int32_t> lat[3];
  int64_t L[3] = { 0, 0, 0 };
  bool lattice = false;
  const char* pe = variant("AFEM_FUNCTOR_PLAN");
  const bool force_slices = pe && std::string(pe) == "slices";
  if (!force_slices && m.dim == 3 && m.nv == 4) {
    if (m.st.valid && m.st.dim == 3) {
      L[0] = m.st.n + 1;
      L[1] = m.st.n + 1;
      L[2] = m.st.k1 - m.st.k0;
      if (L[0] * L[1] * L[2] == n_rows) {
        for (auto& a : lat) a.alloc(n_rows);
        hipLaunchKernelGGL(k_gen_lattice, dim3(grid_for(n_rows, 256)), dim3(256), 0, ctx.stream, n_rows, L[0], L[1],
                           lat[0].p, lat[1].p, lat[2].p);
        AFEM_LAUNCHED();
        lattice = true;
      }
    }
    else if (s.lattice) {
      lattice = lattice_coords(ctx, m, n_rows, lat, L);
    }
  }

  DevBuf<int64_t> nc_ptr;
  DevBuf<int32_t> nc;
  node_cell_adjacency(ctx, m, n_rows, nc_ptr, nc);
  DevBuf<int32_t> r_unit, r_li, err;
  r_unit.alloc(n_rows);
  r_li.alloc(n_rows);
  err.alloc(1);

  std::vector<int32_t> clpos;  // non-lattice plans: the clusters' position -> row map
  for (int attempt = 0; attempt < 2; ++attempt) {
    UnitGeom g{};
    g.nv = m.nv;
    g.n_own = n_rows;
    if (lattice && attempt == 0) {
      // footprints: two layers of fx*fy rows x W k^2 blocks in LDS
      g.lattice = 1;
      g.fx = 8;
      g.fy = k == 1 ? 8 : 4;
      if (k == 3) g.fx = 4;
      // footprint overrides (measurements): fx * fy block rows per layer (one
      // lane each), at most 64
      g.fx = (int)std::max<int64_t>(1, env_int("AFEM_FUNCTOR_FX", g.fx));
      g.fy = (int)std::max<int64_t>(1, env_int("AFEM_FUNCTOR_FY", g.fy));
      if (g.fx * g.fy > 64) throw Error(AFEM_ERR_ARG, "functor plan: AFEM_FUNCTOR_FX * FY exceeds 64 rows");
      g.Lx = L[0];
      g.Ly = L[1];
      g.Lz = L[2];
      g.tx = (L[0] + g.fx - 1) / g.fx;
      g.ty = (L[1] + g.fy - 1) / g.fy;
      const int64_t cols_n = g.tx * g.ty;
      const int64_t target = env_int("AFEM_FUNCTOR_UNITS", 16384);
      const int64_t ns_want = std::max<int64_t>(1, (target + cols_n - 1) / cols_n);
      int64_t zs = env_int("AFEM_FUNCTOR_ZS", (g.Lz + ns_want - 1) / ns_want);
      zs = std::max<int64_t>(4, std::min<int64_t>(zs, 255));
      zs = std::min<int64_t>(zs, g.Lz);
      g.zs = (int)zs;
      g.ns = (g.Lz + zs - 1) / zs;
      g.rl = g.fx * g.fy;
      P.n_units = cols_n * g.ns;
      P.n_stages = cols_n * g.Lz;
      P.nbuf = 2;
    }
    else {
      g.lattice = 0;
      g.rl = 64 / (k * k);
      g.zs = 1;
      const char* ce = variant("AFEM_FUNCTOR_CLUSTER");
      if (!(ce && atoi(ce) == 0)) {
        // breadth-first clusters of rl rows seeded in the processing order
        clpos = cluster_positions(ctx, s, g.rl, P.n_units);
      }
      else {
        // 64 / k^2 rows per piece of the processing order: the last piece may
        // be partial (k = 3: 7 rows, 64 positions per slice are 9 pieces and
        // one row of the next)
        clpos.clear();
        P.n_units = (s.n_slices * 64 + g.rl - 1) / g.rl;
      }
      P.n_stages = P.n_units;
      P.nbuf = 1;
    }
    P.lattice = g.lattice;
    P.rl = g.rl;
    P.fx = g.fx;
    P.fy = g.fy;
    P.zs = g.zs;
    P.layer_rows.alloc((size_t)P.n_stages * g.rl);
    AFEM_HIP(hipMemsetAsync(P.layer_rows.p, 0xFF, P.layer_rows.bytes(), ctx.stream));
    if (g.lattice) {
      hipLaunchKernelGGL(k_rowmap_lattice, dim3(grid_for(n_rows, 256)), dim3(256), 0, ctx.stream, n_rows, lat[0].p,
                         lat[1].p, lat[2].p, g, r_unit.p, r_li.p, P.layer_rows.p);
    }
    else if (!clpos.empty()) {
      DevBuf<int32_t> dpos;
      dpos.alloc(clpos.size());
      AFEM_HIP(hipMemcpyAsync(dpos.p, clpos.data(), clpos.size() * 4, hipMemcpyHostToDevice, ctx.stream));
      hipLaunchKernelGGL(k_rowmap_positions, dim3(grid_for((int64_t)clpos.size(), 256)), dim3(256), 0, ctx.stream,
                         (int64_t)clpos.size(), dpos.p, g.rl, r_unit.p, r_li.p, P.layer_rows.p);
      AFEM_LAUNCHED();
      ctx.sync();
    }
    else {
      hipLaunchKernelGGL(k_rowmap_slices, dim3(grid_for(s.n_slices * 64, 256)), dim3(256), 0, ctx.stream,
                         s.n_slices * 64, s.perm.p, g.rl, r_unit.p, r_li.p, P.layer_rows.p);
    }
    AFEM_LAUNCHED();
    bool span_ok = true;
    if (m.nv == 4)
      build_entries<4>(ctx, b, g, nc_ptr, nc, r_unit, r_li, err, span_ok);
    else
      build_entries<3>(ctx, b, g, nc_ptr, nc, r_unit, r_li, err, span_ok);
    if (!span_ok) continue;  // a cell spans more than two layers: slice pieces
    P.units.alloc(P.n_units);
    const int runs_ok = (k == 1 && g.rl == 64 && g.fx == 8) ? 1 : 0;
    hipLaunchKernelGGL(k_units, dim3(grid_for(P.n_units, 256)), dim3(256), 0, ctx.stream, P.n_units, g,
                       P.layer_rows.p, runs_ok, P.units.p);
    AFEM_LAUNCHED();
    DevBuf<unsigned long long> nf;
    nf.alloc(1);
    AFEM_HIP(hipMemsetAsync(nf.p, 0, nf.bytes(), ctx.stream));
    hipLaunchKernelGGL(k_count_flags, dim3(grid_for(P.n_units, 256)), dim3(256), 0, ctx.stream, P.n_units, P.units.p,
                       nf.p);
    AFEM_LAUNCHED();
    unsigned long long hn = 0;
    AFEM_HIP(hipMemcpyAsync(&hn, nf.p, sizeof(hn), hipMemcpyDeviceToHost, ctx.stream));
    ctx.sync();
    P.n_coalesced = (int64_t)hn;
    P.valid = true;
    return;
  }
  throw Error(AFEM_ERR_STATE, "functor plan: no unit layout");
}

}  // namespace afem
