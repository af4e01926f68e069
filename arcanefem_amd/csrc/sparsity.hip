// One-time structure build on the GPU (replaces BSRFormat::computeSparsity,
// femutils/BSRFormat.h:583-781).
//
// The reference sorts 6*Ncell packed u64 edge keys (K1/K2), counts unique
// edges with atomics (K3), scans (K4) and fills columns with an atomic cursor
// (K5, run-dependent column order).  At 1e8 DoF the edge keys alone are
// 28.6 GB.  Here the structure is built row-locally from a node->cell
// adjacency instead, so the largest temporary is the 4*Ncell incidence list:
//
//   1. count incidences per owned node (int atomics) -> scan -> fill -> sort
//      each node's cell list (deterministic order);
//   2. per row, the sorted unique union of its cells' nodes = the row's
//      columns (diagonal included); count -> scan -> fill;
//   3. the row-local incidence table used by the assembly kernels: for every
//      (row, incident cell) the row-slots of the cell's other nodes packed in
//      one uint32 (8 bits per slot, diagonal slot in the top byte), stored as
//      sliced ELLPACK with slice height 64 = one wavefront, 4 consecutive
//      incidences of a row packed per lane, so a wave reads one coalesced
//      1-KiB line (a 16-B load per lane) per 4 incidence steps.
#include "afem_internal.hpp"

#include <hipcub/hipcub.hpp>

#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <string>

namespace afem {
namespace {

constexpr uint32_t kPad = 0xFFFFFFFFu;
constexpr int kRowCap = 255;  // slots are 8-bit; 0xFF is the padding marker

inline unsigned grid_for(int64_t n, int threads) { return (unsigned)((n + threads - 1) / threads); }

__global__ void k_count_incidence(int64_t n_entries, const int32_t* __restrict__ cn, int64_t n_rows,
                                  int32_t* __restrict__ cnt)
{
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_entries) return;
  int32_t node = cn[t];
  if (node < n_rows) atomicAdd(&cnt[node], 1);
}

__global__ void k_fill_incidence(int64_t n_cells, int nv, const int32_t* __restrict__ cn, int64_t n_rows,
                                 const int64_t* __restrict__ nc_ptr, int32_t* __restrict__ cursor,
                                 int32_t* __restrict__ nc)
{
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_cells * nv) return;
  int64_t cell = t / nv;
  int32_t node = cn[t];
  if (node < n_rows) {
    int pos = atomicAdd(&cursor[node], 1);
    nc[nc_ptr[node] + pos] = (int32_t)cell;
  }
}

// Insertion sort of each node's incident-cell list (short lists).
__global__ void k_sort_lists(int64_t n_rows, const int64_t* __restrict__ ptr, int32_t* __restrict__ v)
{
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rows) return;
  int64_t b = ptr[r], e = ptr[r + 1];
  for (int64_t i = b + 1; i < e; ++i) {
    int32_t key = v[i];
    int64_t j = i - 1;
    while (j >= b && v[j] > key) {
      v[j + 1] = v[j];
      --j;
    }
    v[j + 1] = key;
  }
}

// Sorted unique union of the nodes of a row's incident cells.  One thread per
// row, the row's list in LDS laid out [slot][thread] (bank-conflict free for
// any per-thread slot).  WRITE=false: row length (or -1 if > kRowCap);
// WRITE=true: columns + diagonal position.
constexpr int kUnionThreads = 64;
template <bool WRITE>
__global__ __launch_bounds__(kUnionThreads) void k_row_union(int64_t n_rows, int nv, const int32_t* __restrict__ cn,
                                                             const int64_t* __restrict__ nc_ptr,
                                                             const int32_t* __restrict__ nc,
                                                             int32_t* __restrict__ row_len,
                                                             const int64_t* __restrict__ row_ptr,
                                                             int32_t* __restrict__ cols, int64_t* __restrict__ diag_pos)
{
  __shared__ int32_t buf[(kRowCap + 1) * kUnionThreads];
  const int tid = threadIdx.x;
  int64_t r = (int64_t)blockIdx.x * kUnionThreads + tid;
  if (r >= n_rows) return;
  int m = 1;
  buf[tid] = (int32_t)r;
  bool overflow = false;
  for (int64_t q = nc_ptr[r]; q < nc_ptr[r + 1] && !overflow; ++q) {
    const int32_t* nodes = cn + (int64_t)nc[q] * nv;
    for (int a = 0; a < nv; ++a) {
      int32_t x = nodes[a];
      // binary search in buf[0..m)
      int lo = 0, hi = m;
      while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (buf[mid * kUnionThreads + tid] < x)
          lo = mid + 1;
        else
          hi = mid;
      }
      if (lo < m && buf[lo * kUnionThreads + tid] == x) continue;
      if (m == kRowCap) {
        overflow = true;
        break;
      }
      for (int k = m; k > lo; --k) buf[k * kUnionThreads + tid] = buf[(k - 1) * kUnionThreads + tid];
      buf[lo * kUnionThreads + tid] = x;
      ++m;
    }
  }
  if (!WRITE) {
    row_len[r] = overflow ? -1 : m;
  }
  else {
    int64_t base = row_ptr[r];
    for (int k = 0; k < m; ++k) {
      int32_t c = buf[k * kUnionThreads + tid];
      cols[base + k] = c;
      if (c == (int32_t)r) diag_pos[r] = base + k;
    }
  }
}

__global__ void k_check_len(int64_t n_rows, const int32_t* __restrict__ row_len, int32_t* __restrict__ flags)
{
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rows) return;
  int32_t l = row_len[r];
  if (l < 0) atomicOr(&flags[0], 1);
  else atomicMax(&flags[1], l);
}

// Processing order of a structured box of nodes (the owned nodes of a
// generated mesh are numbered lexicographically, i fastest, in an
// ax x ay x az box): bricks of 4x4x4 nodes (8x8 in 2D) in lexicographic
// brick order, one brick per slice, lane = position in the brick.
__global__ void k_perm_bricks(int64_t n_slices, int dim, int64_t ax, int64_t ay, int64_t az, int32_t* __restrict__ perm)
{
  int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_slices * 64) return;
  const int64_t s = p >> 6;
  const int lane = (int)(p & 63);
  const int bx = dim == 3 ? 4 : 8, by = bx, bz = dim == 3 ? 4 : 1;
  const int64_t nbx = (ax + bx - 1) / bx, nby = (ay + by - 1) / by;
  const int64_t ib = s % nbx, jb = (s / nbx) % nby, kb = s / (nbx * nby);
  const int64_t i = ib * bx + lane % bx;
  const int64_t j = jb * by + (lane / bx) % by;
  const int64_t k = kb * bz + lane / (bx * by);
  perm[p] = (i < ax && j < ay && k < az) ? (int32_t)(i + ax * (j + ay * k)) : -1;
}

// 3D structured boxes, boundary-aware: the interior nodes [1, a-2]^3 in 4x4x4
// bricks (partial bricks at the upper end: idle lanes), then the six boundary
// faces without their box edges in 8x8 tiles, the twelve box edges without
// their corners in runs of 32 (a run's slice then couples ~136 nodes: within
// the block-3 workgroup kernel's 256) and the eight corners one slice each.  Every
// slice then holds rows of one local topology: interior bricks share the
// uniform assembly instance, each face its own, and the box edges / corners
// no longer spoil a face tile (so no face tile falls back to the general
// list; only the few edge and corner slices do).
struct FaceTiles {
  static constexpr int kMaxSeg = 26;  // 6 faces + 12 edges + 8 corners
  int64_t n_core, nbx, nby;
  int nseg;
  int64_t start[kMaxSeg + 1];  // first slice of segment g (start[nseg] = n_slices)
  int64_t U[kMaxSeg], V[kMaxSeg], tu[kMaxSeg], o[kMaxSeg][3];
  int8_t au[kMaxSeg], av[kMaxSeg], tw[kMaxSeg];  // u / v axes; tile width along u (8 faces, 32 edges)
};

__host__ __device__ inline FaceTiles face_tiles(int64_t ax, int64_t ay, int64_t az)
{
  FaceTiles F{};
  const int64_t a[3] = { ax, ay, az };
  const int64_t c[3] = { ax > 2 ? ax - 2 : 0, ay > 2 ? ay - 2 : 0, az > 2 ? az - 2 : 0 };
  F.nbx = (c[0] + 3) / 4;
  F.nby = (c[1] + 3) / 4;
  F.n_core = F.nbx * F.nby * ((c[2] + 3) / 4);
  int64_t acc = F.n_core;
  auto add = [&](int64_t U, int64_t V, int tw, int64_t o0, int64_t o1, int64_t o2, int au, int av) {
    if (U <= 0 || V <= 0) return;
    const int g = F.nseg++;
    F.U[g] = U;
    F.V[g] = V;
    F.tw[g] = (int8_t)tw;
    F.tu[g] = (U + tw - 1) / tw;
    F.o[g][0] = o0;
    F.o[g][1] = o1;
    F.o[g][2] = o2;
    F.au[g] = (int8_t)au;
    F.av[g] = (int8_t)av;
    F.start[g] = acc;
    acc += F.tu[g] * ((V + 64 / tw - 1) / (64 / tw));
  };
  // the ends of axis d: one plane when the box is one node thick along d
  auto n_end = [&](int d) { return a[d] > 1 ? 2 : 1; };
  auto end = [&](int d, int e) { return e ? a[d] - 1 : (int64_t)0; };
  for (int d = 2; d >= 0; --d) {  // faces: k planes, j planes, i planes; u, v = the other axes, lower first
    const int u = d == 0 ? 1 : 0, v = d == 2 ? 1 : 2;
    for (int e = 0; e < n_end(d); ++e) {
      int64_t o[3] = { 1, 1, 1 };
      o[d] = end(d, e);
      add(c[u], c[v], 8, o[0], o[1], o[2], u, v);
    }
  }
  for (int d = 0; d < 3; ++d) {  // edges along d
    const int p = d == 0 ? 1 : 0, q = d == 2 ? 1 : 2;
    for (int eq = 0; eq < n_end(q); ++eq)
      for (int ep = 0; ep < n_end(p); ++ep) {
        int64_t o[3];
        o[d] = 1;
        o[p] = end(p, ep);
        o[q] = end(q, eq);
        add(c[d], 1, 32, o[0], o[1], o[2], d, d);
      }
  }
  for (int ek = 0; ek < n_end(2); ++ek)  // corners
    for (int ej = 0; ej < n_end(1); ++ej)
      for (int ei = 0; ei < n_end(0); ++ei) add(1, 1, 64, end(0, ei), end(1, ej), end(2, ek), 0, 0);
  F.start[F.nseg] = acc;
  return F;
}

__global__ void k_perm_bricks_bd(int64_t n_slices, int64_t ax, int64_t ay, int64_t az, FaceTiles F,
                                 int32_t* __restrict__ perm)
{
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_slices * 64) return;
  const int64_t s = p >> 6;
  const int lane = (int)(p & 63);
  int64_t i = -1, j = -1, k = -1;
  if (s < F.n_core) {
    const int64_t ib = s % F.nbx, jb = (s / F.nbx) % F.nby, kb = s / (F.nbx * F.nby);
    i = 1 + 4 * ib + (lane & 3);
    j = 1 + 4 * jb + ((lane >> 2) & 3);
    k = 1 + 4 * kb + (lane >> 4);
    if (i > ax - 2 || j > ay - 2 || k > az - 2) i = -1;
  }
  else {
    int g = 0;
    while (g + 1 < F.nseg && s >= F.start[g + 1]) ++g;
    const int64_t t = s - F.start[g];
    const int tw = F.tw[g];
    const int64_t u = tw * (t % F.tu[g]) + lane % tw, v = (64 / tw) * (t / F.tu[g]) + lane / tw;
    if (u < F.U[g] && v < F.V[g]) {
      int64_t x[3] = { F.o[g][0], F.o[g][1], F.o[g][2] };
      x[F.au[g]] += u;
      x[F.av[g]] += v;  // lines and corners: v = 0
      i = x[0];
      j = x[1];
      k = x[2];
    }
  }
  perm[p] = i >= 0 ? (int32_t)(i + ax * (j + ay * k)) : -1;
}

__global__ void k_count_valid(int64_t n, const int32_t* __restrict__ perm, unsigned long long* __restrict__ out)
{
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned long long b = __ballot(p < n && perm[p] >= 0);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(out, (unsigned long long)__popcll(b));
}

// Meshes without a structured numbering: the processing order sorts the
// owned nodes along a Hilbert curve of their coordinates, so the 64
// rows of a slice are spatial neighbours (few distinct coupled nodes: the LDS
// coordinate cache stays small, gathers stay in L2) whatever the caller's
// numbering.  The matrix itself stays in the caller's node order.
__device__ __forceinline__ unsigned long long ordered_bits(double v)
{
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double from_ordered_bits(unsigned long long u)
{
  return __longlong_as_double((long long)((u >> 63) ? (u & 0x7fffffffffffffffull) : ~u));
}
__global__ void k_bbox(int64_t n, const double* __restrict__ coords, unsigned long long* __restrict__ box)
{
  unsigned long long mn[3] = { ~0ull, ~0ull, ~0ull }, mx[3] = { 0ull, 0ull, 0ull };
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    for (int a = 0; a < 3; ++a) {
      const unsigned long long u = ordered_bits(coords[3 * i + a]);
      mn[a] = u < mn[a] ? u : mn[a];
      mx[a] = u > mx[a] ? u : mx[a];
    }
  for (int a = 0; a < 3; ++a) {
    atomicMin(box + a, mn[a]);
    atomicMax(box + 3 + a, mx[a]);
  }
}
__device__ __forceinline__ uint64_t spread3(uint64_t v)  // 21 bits -> every third bit
{
  v &= 0x1fffffull;
  v = (v | v << 32) & 0x1f00000000ffffull;
  v = (v | v << 16) & 0x1f0000ff0000ffull;
  v = (v | v << 8) & 0x100f00f00f00f00full;
  v = (v | v << 4) & 0x10c30c30c30c30c3ull;
  v = (v | v << 2) & 0x1249249249249249ull;
  return v;
}
// Hilbert index of a point of the 2^21-grid (Skilling's transpose algorithm:
// undo the excess work, Gray-encode, interleave the transposed bits): unlike
// the Morton curve it has no jumps, so 64 consecutive nodes form a compact
// cluster (fewer coupled nodes per slice).
__device__ __forceinline__ uint64_t hilbert3(uint32_t x, uint32_t y, uint32_t z)
{
  uint32_t X[3] = { x, y, z };
  const uint32_t M = 1u << 20;
  for (uint32_t Q = M; Q > 1; Q >>= 1) {
    const uint32_t P = Q - 1;
    for (int i = 0; i < 3; ++i) {
      if (X[i] & Q) {
        X[0] ^= P;
      }
      else {
        const uint32_t t = (X[0] ^ X[i]) & P;
        X[0] ^= t;
        X[i] ^= t;
      }
    }
  }
  X[1] ^= X[0];
  X[2] ^= X[1];
  uint32_t t = 0;
  for (uint32_t Q = M; Q > 1; Q >>= 1)
    if (X[2] & Q) t ^= Q - 1;
  for (int i = 0; i < 3; ++i) X[i] ^= t;
  return spread3(X[0]) << 2 | spread3(X[1]) << 1 | spread3(X[2]);
}
// curve keys of the owned nodes: HILBERT (default) or Morton (AFEM_ORDER=morton)
template <bool HILBERT>
__global__ void k_curve_keys(int64_t n, const double* __restrict__ coords, const unsigned long long* __restrict__ box,
                             uint64_t* __restrict__ keys, int32_t* __restrict__ ids)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t q[3];
  for (int a = 0; a < 3; ++a) {
    const double lo = from_ordered_bits(box[a]), hi = from_ordered_bits(box[3 + a]);
    const double t = hi > lo ? (coords[3 * i + a] - lo) / (hi - lo) : 0.0;
    q[a] = (uint32_t)fmin(fmax(t * 2097151.0, 0.0), 2097151.0);
  }
  keys[i] = HILBERT ? hilbert3(q[0], q[1], q[2]) : (spread3(q[0]) | spread3(q[1]) << 1 | spread3(q[2]) << 2);
  ids[i] = (int32_t)i;
}
__global__ void k_perm_from_sorted(int64_t n_pos, int64_t n_rows, const int32_t* __restrict__ sorted,
                                   int32_t* __restrict__ perm)
{
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n_pos) perm[p] = p < n_rows ? sorted[p] : -1;
}

__global__ void k_perm_identity(int64_t n_pos, int64_t n_rows, int32_t* __restrict__ perm)
{
  int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n_pos) perm[p] = p < n_rows ? (int32_t)p : -1;
}

// ---- lattice recovery (meshes that arrive as arrays): when the owned nodes
// of a tetrahedral mesh sit on a (jittered) lattice -- a structured box in any
// numbering, e.g. the caller's own or a random one -- the processing order is
// the brick order of that lattice, so the uniform / stencil instances apply as
// they do to the generator's boxes.  Per axis the owned nodes' coordinates are
// sorted and cut into layers at the gaps wider than half the widest gap (within
// a layer the jitter spread is < 0.2 h, between layers > 0.8 h); the layer
// counts must multiply to the owned node count and every lattice point must
// hold exactly one node.  Only the ORDER depends on this: strips, signatures
// and bank placement are computed from the real connectivity afterwards, so a
// wrong guess costs speed, never values.
__global__ void k_axis_keys(int64_t n, const double* __restrict__ coords, int a, uint64_t* __restrict__ keys,
                            int32_t* __restrict__ ids)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  keys[i] = (uint64_t)ordered_bits(coords[3 * i + a]);
  ids[i] = (int32_t)i;
}
__global__ void k_max_gap(int64_t n, const uint64_t* __restrict__ sorted, unsigned long long* __restrict__ out)
{
  double g = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n; i += (int64_t)gridDim.x * blockDim.x)
    g = fmax(g, from_ordered_bits(sorted[i + 1]) - from_ordered_bits(sorted[i]));
  atomicMax(out, (unsigned long long)__double_as_longlong(g));  // g >= 0: the bits order like the values
}
__global__ void k_gap_flags(int64_t n, const uint64_t* __restrict__ sorted, double thr,
                            int32_t* __restrict__ flag)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  flag[i] = (i + 1 < n && from_ordered_bits(sorted[i + 1]) - from_ordered_bits(sorted[i]) > thr) ? 1 : 0;
}
// layer of sorted position i = number of layer boundaries before it
__global__ void k_layer_scatter(int64_t n, const int32_t* __restrict__ ids, const int64_t* __restrict__ scan,
                                int32_t* __restrict__ layer)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) layer[ids[i]] = (int32_t)scan[i];
}
__global__ void k_lattice_fill(int64_t n, const int32_t* __restrict__ lx, const int32_t* __restrict__ ly,
                               const int32_t* __restrict__ lz, int64_t Lx, int64_t Ly, int32_t* __restrict__ lat,
                               int32_t* __restrict__ bad)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t c = lx[i] + Lx * (ly[i] + Ly * (int64_t)lz[i]);
  if (atomicCAS(lat + c, -1, (int32_t)i) != -1) *bad = 1;
}
__global__ void k_perm_map(int64_t n_pos, const int32_t* __restrict__ lat, int32_t* __restrict__ perm)
{
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n_pos && perm[p] >= 0) perm[p] = lat[perm[p]];
}

// Per slice: the max incidence count (ELL width, rounded up to a multiple of
// 4) and the table size.
__global__ void k_slice_width(int64_t n_slices, const int32_t* __restrict__ perm, const int64_t* __restrict__ nc_ptr,
                              int32_t* __restrict__ slice_k, int64_t* __restrict__ slice_sz)
{
  int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_slices) return;
  int64_t w = 0;
  for (int l = 0; l < 64; ++l) {
    const int32_t r = perm[s * 64 + l];
    if (r < 0) continue;
    const int64_t c = nc_ptr[r + 1] - nc_ptr[r];
    w = c > w ? c : w;
  }
  w = (w + 3) & ~(int64_t)3;  // groups of 4 incidences per lane (one 16-B load)
  slice_k[s] = (int32_t)w;
  slice_sz[s] = w * 64;
}

__device__ int find_slot(const int32_t* c, int len, int32_t x)
{
  int lo = 0, hi = len;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (c[mid] < x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

__global__ void k_fill_inc(int64_t n_pos, int nv, const int32_t* __restrict__ perm, const int32_t* __restrict__ cn,
                           const int64_t* __restrict__ nc_ptr, const int32_t* __restrict__ nc,
                           const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ cols,
                           const int64_t* __restrict__ slice_ptr, const int32_t* __restrict__ slice_k,
                           uint32_t* __restrict__ inc)
{
  int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pos) return;
  const int64_t s = p >> 6;
  const int lane = (int)(p & 63);
  uint32_t* out = inc + slice_ptr[s] + lane * 4;  // entry k at (k/4)*256 + lane*4 + k%4
  const int32_t r = perm[p];
  int cnt = 0;
  if (r >= 0) {
    const int32_t* c = cols + row_ptr[r];
    const int len = (int)(row_ptr[r + 1] - row_ptr[r]);
    const uint32_t dslot = (uint32_t)find_slot(c, len, r);
    const int64_t b = nc_ptr[r];
    cnt = (int)(nc_ptr[r + 1] - b);
    for (int k = 0; k < cnt; ++k) {
      const int32_t* nodes = cn + (int64_t)nc[b + k] * nv;
      uint32_t packed = dslot << 24;
      int o = 0;
      for (int a = 0; a < nv; ++a) {
        int32_t x = nodes[a];
        if (x == r) continue;
        packed |= (uint32_t)find_slot(c, len, x) << (8 * o);
        ++o;
      }
      if (nv == 3) packed |= 0xFFu << 16;  // unused third slot
      out[(int64_t)(k >> 2) * 256 + (k & 3)] = packed;
    }
  }
  for (int k = cnt; k < slice_k[s]; ++k) out[(int64_t)(k >> 2) * 256 + (k & 3)] = kPad;
}

// Slice node lists.  One wavefront per slice: the columns of the slice's
// rows are bitonic-sorted in LDS and made unique (ballot compaction); the
// WRITE pass stores the list and, for every (slot, lane), the column's
// index in it.  Pass 1 (WRITE = false) only records the slice width and the
// list length, for the prefix sums.
template <bool WRITE>
__global__ __launch_bounds__(64) void k_slice_nodes(const int32_t* __restrict__ perm, const int64_t* __restrict__ row_ptr,
                                                    const int32_t* __restrict__ cols, int32_t* __restrict__ slice_w,
                                                    int64_t* __restrict__ slice_nu, const int64_t* __restrict__ snode_ptr,
                                                    int32_t* __restrict__ snode, const int64_t* __restrict__ lidx_ptr,
                                                    uint16_t* __restrict__ lidx)
{
  extern __shared__ int32_t buf[];
  const int lane = threadIdx.x;
  const int64_t s = blockIdx.x;
  const int32_t r = perm[s * 64 + lane];
  const int64_t rb = r >= 0 ? row_ptr[r] : 0;
  const int len = r >= 0 ? (int)(row_ptr[r + 1] - rb) : 0;
  int W = len;
  for (int o = 32; o > 0; o >>= 1) W = max(W, __shfl_xor(W, o));
  int M = 64;
  while (M < 64 * W) M <<= 1;
  for (int t = 0; t < (M >> 6); ++t) buf[t * 64 + lane] = t < len ? cols[rb + t] : INT_MAX;
  __syncthreads();
  for (int k = 2; k <= M; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = lane; i < M; i += 64) {
        const int q = i ^ j;
        if (q > i) {
          const int a = buf[i], b = buf[q];
          if ((a > b) == ((i & k) == 0)) {
            buf[i] = b;
            buf[q] = a;
          }
        }
      }
      __syncthreads();
    }
  int cnt = 0, carry = -1;
  for (int base = 0; base < 64 * W; base += 64) {
    const int v = buf[base + lane];
    int prev = __shfl_up(v, 1);
    if (lane == 0) prev = carry;
    carry = __shfl(v, 63);
    const bool f = v != INT_MAX && v != prev;
    const unsigned long long m = __ballot(f);
    const int pos = cnt + __popcll(m & ((1ull << lane) - 1ull));
    __syncthreads();
    if (f) buf[pos] = v;  // pos <= base + lane: later chunks are untouched
    cnt += __popcll(m);
    __syncthreads();
  }
  if (!WRITE) {
    if (lane == 0) {
      slice_w[s] = W;
      slice_nu[s] = cnt;
    }
    return;
  }
  const int64_t u0 = snode_ptr[s];
  for (int u = lane; u < cnt; u += 64) snode[u0 + u] = buf[u];
  const int64_t l0 = lidx_ptr[s];
  for (int t = 0; t < W; ++t) {
    uint16_t v = 0;
    if (t < len) v = (uint16_t)find_slot(buf, cnt, cols[rb + t]);
    lidx[l0 + (int64_t)t * 64 + lane] = v;
  }
}

__global__ void k_times64(int64_t n, const int32_t* __restrict__ w, int64_t* __restrict__ out)
{
  int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s < n) out[s] = 64 * (int64_t)w[s];
}

__global__ void k_slice_max(int64_t n_slices, const int32_t* __restrict__ perm, const int64_t* __restrict__ row_ptr,
                            const int32_t* __restrict__ slice_w, const int64_t* __restrict__ slice_nu,
                            const int32_t* __restrict__ slice_k, unsigned long long* __restrict__ out)
{
  int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_slices) return;
  unsigned long long seg = 0;
  for (int l = 0; l < 64; ++l) {
    const int32_t r = perm[s * 64 + l];
    if (r >= 0) seg += (unsigned long long)(row_ptr[r + 1] - row_ptr[r]);
  }
  atomicMax(&out[0], seg);
  atomicMax(&out[1], (unsigned long long)slice_w[s]);
  atomicMax(&out[2], (unsigned long long)slice_nu[s]);
  atomicMax(&out[3], (unsigned long long)slice_k[s]);
}

// ---------------------------------------------------------------- row strips
// Around a row node r the incident cells form a star; its link is a
// triangulated surface (tets: triangles of the other three nodes) or a path /
// cycle (triangles: edges of the other two nodes).  A strip orders cells so
// that consecutive ones share a face through r: the window of the last NV-1
// other nodes advances by ONE new node per cell, either dropping its oldest
// node ("shift", kind 0) or its middle one ("swap", kind 1).  The assembly
// kernel then gathers one node per cell instead of NV-1 and reuses one
// cofactor (cross product) of the previous cell.  Stream byte = slot (6 bits,
// position of the node in the row's columns) | kind << 6; kind 2 = priming
// node (window fill at a strip start, no cell), kind 3 = padding (slot = the
// row's diagonal: a zero vector, no cell).
// Greedy cover (deterministic): start at the unvisited link triangle with the
// fewest unvisited neighbours, try the NV-1 choices of the "newest" node,
// extend with the candidate having the fewest unvisited neighbours (shift
// before swap), keep the longest extension.  Kuhn boxes: one strip per row
// (steps = cells + 2); unstructured golden meshes: 1.1-1.25 steps per cell.
constexpr int kStripMaxCells = 64;  // link elements per row (64-bit masks)
constexpr int kStripMaxSlots = 64;  // 6-bit slots

struct StripScratch {
  uint64_t mask[kStripMaxCells];  // slots of each link element
  uint64_t adj[kStripMaxCells];   // link elements sharing NV-2 slots (an edge / a node)
  uint8_t sl[kStripMaxCells][3];
};

// greedy extension from window (w0,w1,w2) [tets] / (w1,w2) [triangles] over `unv`;
// returns the number of cells appended; emits bytes if out != nullptr
__device__ int strip_extend(const StripScratch& S, int k, int cur, uint64_t unv, int w0, int w1, int w2,
                            uint8_t* out, uint64_t* unv_out)
{
  int n = 0;
  for (;;) {
    uint64_t cand = S.adj[cur] & unv;
    int best = -1, best_kind = 0, best_key = 1 << 30;
    while (cand) {
      const int u = __ffsll((long long)cand) - 1;
      cand &= cand - 1;
      const uint64_t mu = S.mask[u];
      int kind = -1;
      if (k == 3) {
        if ((mu >> w1 & 1) && (mu >> w2 & 1)) kind = 0;
        else if ((mu >> w0 & 1) && (mu >> w2 & 1)) kind = 1;
      }
      else {
        if (mu >> w2 & 1) kind = 0;
        else if (mu >> w1 & 1) kind = 1;
      }
      if (kind < 0) continue;
      const int key = (__popcll(S.adj[u] & unv & ~(1ull << u)) << 3) | (kind << 2);
      if (key < best_key) {
        best_key = key;
        best = u;
        best_kind = kind;
      }
    }
    if (best < 0) break;
    unv &= ~(1ull << best);
    // the new node: the element's slot not in the kept part of the window
    int d = -1;
    for (int a = 0; a < k; ++a) {
      const int x = S.sl[best][a];
      const bool kept = (k == 3) ? (best_kind == 0 ? (x == w1 || x == w2) : (x == w0 || x == w2))
                                 : (best_kind == 0 ? x == w2 : x == w1);
      if (!kept) d = x;
    }
    if (out) out[n] = (uint8_t)(d | (best_kind << 6));
    ++n;
    if (k == 3) {
      if (best_kind == 0) w0 = w1;
      w1 = w2;
      w2 = d;
    }
    else {
      if (best_kind == 0) w1 = w2;
      w2 = d;
    }
    cur = best;
  }
  if (unv_out) *unv_out = unv;
  return n;
}

// One thread per processing position.  WRITE = false: stream length (or -1
// when the row does not fit the 6-bit slot / 64-cell limits); WRITE = true:
// the stream into the sliced layout (16 steps per 16-B chunk per lane) and
// the row's diagonal slot.
template <bool WRITE>
__global__ __launch_bounds__(64) void k_strip_rows(int64_t n_pos, int nv, const int32_t* __restrict__ perm,
                                                   const int32_t* __restrict__ cn, const int64_t* __restrict__ nc_ptr,
                                                   const int32_t* __restrict__ nc, const int64_t* __restrict__ row_ptr,
                                                   const int32_t* __restrict__ cols, int32_t* __restrict__ strip_len,
                                                   const int64_t* __restrict__ strip_ptr,
                                                   const int32_t* __restrict__ strip_c, uint8_t* __restrict__ strip,
                                                   uint8_t* __restrict__ dslot_out)
{
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pos) return;
  const int64_t sl = p >> 6;
  const int lane = (int)(p & 63);
  const int32_t r = perm[p];
  const int k = nv - 1;
  int total = 0;
  int dslot = 0;
  uint8_t buf[2 * kStripMaxCells + 16];
  if (r >= 0) {
    const int32_t* c = cols + row_ptr[r];
    const int len = (int)(row_ptr[r + 1] - row_ptr[r]);
    const int64_t b = nc_ptr[r];
    const int T = (int)(nc_ptr[r + 1] - b);
    dslot = find_slot(c, len, r);
    if (len > kStripMaxSlots || T > kStripMaxCells) {
      if (!WRITE) strip_len[p] = -1;
      return;
    }
    StripScratch S;
    for (int t = 0; t < T; ++t) {
      const int32_t* nodes = cn + (int64_t)nc[b + t] * nv;
      uint64_t m = 0;
      int o = 0;
      for (int a = 0; a < nv; ++a) {
        const int32_t x = nodes[a];
        if (x == r) continue;
        const int sx = find_slot(c, len, x);
        S.sl[t][o++] = (uint8_t)sx;
        m |= 1ull << sx;
      }
      S.mask[t] = m;
    }
    for (int t = 0; t < T; ++t) {
      uint64_t a = 0;
      for (int u = 0; u < T; ++u)
        if (u != t && __popcll(S.mask[t] & S.mask[u]) == k - 1) a |= 1ull << u;
      S.adj[t] = a;
    }
    uint64_t unv = T == 64 ? ~0ull : ((1ull << T) - 1);
    while (unv) {
      // start: fewest unvisited neighbours
      int t0 = -1, bk = 1 << 30;
      for (uint64_t q = unv; q; q &= q - 1) {
        const int t = __ffsll((long long)q) - 1;
        const int key = __popcll(S.adj[t] & unv);
        if (key < bk) {
          bk = key;
          t0 = t;
        }
      }
      unv &= ~(1ull << t0);
      // orientation: which node is the newest (must be in the next shared face)
      int best_rot = 0, best_n = -1;
      for (int rot = 0; rot < k; ++rot) {
        int w[3];
        for (int a = 0; a < k; ++a) w[a] = S.sl[t0][(a + rot) % k];
        const int n = k == 3 ? strip_extend(S, k, t0, unv, w[0], w[1], w[2], nullptr, nullptr)
                             : strip_extend(S, k, t0, unv, 0, w[0], w[1], nullptr, nullptr);
        if (n > best_n) {
          best_n = n;
          best_rot = rot;
        }
      }
      int w[3];
      for (int a = 0; a < k; ++a) w[a] = S.sl[t0][(a + best_rot) % k];
      // priming nodes (kind 2) then the start cell (kind 0: shift, emit)
      for (int a = 0; a < k - 1; ++a) buf[total++] = (uint8_t)(w[a] | (2 << 6));
      buf[total++] = (uint8_t)w[k - 1];
      const int n = k == 3 ? strip_extend(S, k, t0, unv, w[0], w[1], w[2], buf + total, &unv)
                           : strip_extend(S, k, t0, unv, 0, w[0], w[1], buf + total, &unv);
      total += n;
    }
  }
  if (!WRITE) {
    strip_len[p] = total;
    return;
  }
  dslot_out[p] = (uint8_t)dslot;
  uint8_t* out = strip + strip_ptr[sl] + lane * 16;
  const int steps = 16 * strip_c[sl];
  for (int j = 0; j < steps; ++j) out[(int64_t)(j >> 4) * 1024 + (j & 15)] = j < total ? buf[j] : (uint8_t)(dslot | (3 << 6));
}

// per position: the row's CSR offset, and its diagonal slot | length << 8 |
// local index of the row node in the slice's node list << 16
__global__ void k_pos_rows(int64_t n_pos, const int32_t* __restrict__ perm, const int64_t* __restrict__ row_ptr,
                           const uint8_t* __restrict__ dslot, const int64_t* __restrict__ lidx_ptr,
                           const uint16_t* __restrict__ lidx, int64_t* __restrict__ pos_rb,
                           uint32_t* __restrict__ pos_dl)
{
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pos) return;
  const int32_t r = perm[p];
  const int64_t b = r >= 0 ? row_ptr[r] : 0;
  const int64_t len = r >= 0 ? row_ptr[r + 1] - b : 0;
  const uint32_t ds = dslot[p];
  const uint32_t u = lidx[lidx_ptr[p >> 6] + 64 * (int64_t)ds + (p & 63)];
  pos_rb[p] = b;
  pos_dl[p] = ds | (uint32_t)len << 8 | (u & 0xFFFFu) << 16;
}

// Companion of the strip stream: for every step byte, the local index (in the
// slice's node list) of the node its slot names, same layout (u8: streams of
// slices with more than 256 nodes are not used by the scalar strip kernels).
__global__ void k_strip_local(int64_t n_pos, const uint8_t* __restrict__ strip, const int64_t* __restrict__ strip_ptr,
                              const int32_t* __restrict__ strip_c, const int64_t* __restrict__ lidx_ptr,
                              const uint16_t* __restrict__ lidx, uint8_t* __restrict__ strip_u)
{
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pos) return;
  const int64_t sl = p >> 6;
  const int lane = (int)(p & 63);
  const int64_t base = strip_ptr[sl] + lane * 16, l0 = lidx_ptr[sl] + lane;
  const int steps = 16 * strip_c[sl];
  for (int j = 0; j < steps; ++j) {
    const int64_t o = base + (int64_t)(j >> 4) * 1024 + (j & 15);
    strip_u[o] = (uint8_t)lidx[l0 + 64 * (int64_t)(strip[o] & 63u)];
  }
}

// LDS-bank-aware placement of a uniform slice's node list (the strip
// kernels' coordinate cache, 24 B per node at position q).  A step's
// coordinate gather is one ds_read2_b64 (x, y: per access four groups of 16
// lanes over 32 banks; 16 nodes at 6-dword stride are conflict-free when their
// positions are distinct mod 16) and one ds_read_b64 (z: two groups of 32
// lanes over 64 banks: distinct mod 32); bank model measured with
// tools/lds_probe.hip.  In a uniform slice every row takes the same
// stencil step at step j, so on a structured brick the node read by lane L at
// step j is "L + d_j" in the brick's lane numbering: a node class
// c(u) = (L + s_j) mod 32, consistent over every (lane, step) reading u, makes
// every gather conflict-free.  This pass finds the shifts s_j (the row's own
// node has shift 0) by propagation over the steps, checks consistency, and
// places node u at q = c(u) + 32 m (m = rank within its class, q < maxq;
// extra nodes fill free positions).  Slices that
// are not uniform, not consistent or larger than 256 nodes keep their order
// (identity).  Positions left free repeat the slice's first node.  Every
// kernel addresses the cache through the remapped local indices, so the
// values do not change.  One wavefront per slice.
// General (non-uniform) slices: every lane reads a node of its own at a step,
// so no shift makes the classes consistent.  A greedy colouring instead: step
// by step, lane by lane, a node read for the first time takes the least-used
// class (with room left below maxq) that no node read at the same step by
// the lanes of its 32-lane half already holds (mod 32: the z read) or, within
// its 16-lane quarter, holds mod 16 (the x, y read); nodes never read take any
// class with room.  Placement as for the uniform slices: q = c + 32 m.
__device__ void bank_place_general(int lane, int nu, int n, bool act, const uint8_t* st, int maxq, int* cls,
                                   int* used, uint8_t* qo, int32_t* nu_out)
{
  for (int u = lane; u < 256; u += 64) cls[u] = -1;
  if (lane < 32) used[lane] = 0;
  __syncthreads();
  auto cap = [&](int c) { return (maxq - c + 31) / 32; };  // positions c + 32 m < maxq
  for (int j = 0; j < n; ++j) {
    const int u = act ? (int)st[(j >> 4) * 1024 + (j & 15)] : -1;
    for (int t = 0; t < 64; ++t) {
      const int ut = __shfl(u, t);
      if (ut < 0) continue;  // wave-uniform
      const int myc = u >= 0 ? cls[u] : -1;
      int bits = 0;
      if (((lane ^ t) & 32) == 0 && lane != t && u >= 0 && u != ut && myc >= 0) {
        bits = 1 << myc;
        if (((lane ^ t) & 16) == 0) bits |= 1 << (myc ^ 16);
      }
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) bits |= __shfl_xor(bits, o);
      if (lane == t && cls[u] < 0) {
        int best = -1, bu = 1 << 30;
        for (int pass = 0; pass < 2 && best < 0; ++pass)
          for (int c = 0; c < 32; ++c)
            if (used[c] < cap(c) && (pass == 1 || !((bits >> c) & 1)) && used[c] < bu) {
              best = c;
              bu = used[c];
            }
        cls[u] = best;
        ++used[best];
      }
      __syncthreads();
    }
  }
  if (lane == 0) {
    uint8_t cnt[32];
    for (int c = 0; c < 32; ++c) cnt[c] = 0;
    int top = -1;
    for (int u = 0; u < nu; ++u) {
      int c = cls[u];
      if (c < 0) {  // never read by a step: any class with room
        int bu = 1 << 30;
        for (int k = 0; k < 32; ++k)
          if (used[k] < cap(k) && used[k] < bu) {
            c = k;
            bu = used[k];
          }
        ++used[c];
      }
      const int q = c + 32 * cnt[c]++;
      qo[u] = (uint8_t)q;
      top = max(top, q);
    }
    for (int u = nu; u < 256; ++u) qo[u] = qo[0];
    *nu_out = top + 1;
  }
}

__global__ __launch_bounds__(64) void k_bank_place(int64_t n_slices, const uint8_t* __restrict__ uflag,
                                                   const int32_t* __restrict__ perm,
                                                   const int64_t* __restrict__ snode_ptr,
                                                   const uint8_t* __restrict__ strip_u,
                                                   const int64_t* __restrict__ strip_ptr,
                                                   const int32_t* __restrict__ strip_n,
                                                   const uint32_t* __restrict__ pos_dl, uint8_t* __restrict__ q_of_u,
                                                   int32_t* __restrict__ nu_new, int maxq, int general)
{
  __shared__ int cls[256];
  __shared__ int shift[32];
  __shared__ int bad;
  const int lane = threadIdx.x;
  const int64_t sl = blockIdx.x;
  if (sl >= n_slices) return;
  const int nu = (int)(snode_ptr[sl + 1] - snode_ptr[sl]);
  uint8_t* qo = q_of_u + sl * 256;
  auto identity = [&]() {
    for (int u = lane; u < 256; u += 64) qo[u] = (uint8_t)(u < nu ? u : 0);
    if (lane == 0) nu_new[sl] = nu;
  };
  const int n = strip_n[sl];
  if (!uflag[sl] && general && nu <= maxq && n <= 32) {
    bank_place_general(lane, nu, n, perm[sl * 64 + lane] >= 0, strip_u + strip_ptr[sl] + lane * 16, maxq, cls,
                       shift, qo, nu_new + sl);
    return;
  }
  if (!uflag[sl] || nu > maxq || n > 32) {
    identity();
    return;
  }
  const bool act = perm[sl * 64 + lane] >= 0;
  const uint8_t* st = strip_u + strip_ptr[sl] + lane * 16;
  const int own = (int)((pos_dl[sl * 64 + lane] >> 16) & 0xFFu);
  for (int u = lane; u < 256; u += 64) cls[u] = -1;
  if (lane < 32) shift[lane] = -1;
  if (lane == 0) bad = 0;
  __syncthreads();
  if (act) cls[own] = lane & 31;
  __syncthreads();
  for (int pass = 0; pass < 32; ++pass) {
    bool progress = false, open = false;
    for (int j = 0; j < n; ++j) {
      if (shift[j] >= 0) continue;
      const int u = st[(j >> 4) * 1024 + (j & 15)];
      const int c = act ? cls[u] : -1;
      const unsigned long long b = __ballot(c >= 0);
      if (!b) {
        open = true;
        continue;
      }
      const int f = __ffsll((long long)b) - 1;
      const int sj = (__shfl(c, f) - f) & 31;
      __syncthreads();
      if (act) {
        const int want = (lane + sj) & 31;
        if (c < 0) cls[u] = want;
      }
      if (lane == 0) shift[j] = sj;
      progress = true;
      __syncthreads();
    }
    if (!open || !progress) break;
  }
  __syncthreads();
  // consistency: every (lane, step) and every row's own node
  bool ok = !act || cls[own] == (lane & 31);
  for (int j = 0; j < n; ++j) {
    const int u = st[(j >> 4) * 1024 + (j & 15)];
    if (act && (shift[j] < 0 || cls[u] != ((lane + shift[j]) & 31))) ok = false;
  }
  if (!ok) atomicOr(&bad, 1);
  __syncthreads();
  if (bad) {
    identity();
    return;
  }
  if (lane == 0) {
    uint8_t cnt[32];
    uint32_t taken[8] = { 0, 0, 0, 0, 0, 0, 0, 0 };
    for (int c = 0; c < 32; ++c) cnt[c] = 0;
    int top = -1;
    for (int u = 0; u < nu; ++u) {
      const int c = cls[u];
      if (c >= 0 && c + 32 * cnt[c] < maxq) {
        const int q = c + 32 * cnt[c]++;
        qo[u] = (uint8_t)q;
        taken[q >> 5] |= 1u << (q & 31);
        top = max(top, q);
        cls[u] = 256;  // placed
      }
    }
    int free_q = 0;
    for (int u = 0; u < nu; ++u) {
      if (cls[u] == 256) continue;
      while (taken[free_q >> 5] >> (free_q & 31) & 1u) ++free_q;
      qo[u] = (uint8_t)free_q;
      taken[free_q >> 5] |= 1u << (free_q & 31);
      top = max(top, free_q);
    }
    for (int u = nu; u < 256; ++u) qo[u] = qo[0];
    nu_new[sl] = top + 1;
  }
}

// new node lists (free positions repeat the slice's first node, never read by a lane)
__global__ __launch_bounds__(64) void k_snode_place(int64_t n_slices, const int64_t* __restrict__ ptr_old,
                                                    const int32_t* __restrict__ snode_old,
                                                    const int64_t* __restrict__ ptr_new, int32_t* __restrict__ snode_new,
                                                    const uint8_t* __restrict__ q_of_u)
{
  const int lane = threadIdx.x;
  const int64_t sl = blockIdx.x;
  if (sl >= n_slices) return;
  const int64_t a = ptr_old[sl], nu = ptr_old[sl + 1] - a, b = ptr_new[sl], nn = ptr_new[sl + 1] - b;
  if (nu > 256) {
    for (int64_t u = lane; u < nu; u += 64) snode_new[b + u] = snode_old[a + u];
    return;
  }
  const int32_t first = nu > 0 ? snode_old[a] : 0;
  for (int64_t q = lane; q < nn; q += 64) snode_new[b + q] = first;
  __syncthreads();
  for (int64_t u = lane; u < nu; u += 64) snode_new[b + q_of_u[sl * 256 + u]] = snode_old[a + u];
}

// renumber the local node indices of the strips, the column-index table and the row positions
__global__ void k_local_place(int64_t n_pos, const int64_t* __restrict__ snode_ptr_old,
                              const uint8_t* __restrict__ q_of_u, uint8_t* __restrict__ strip_u,
                              const int64_t* __restrict__ strip_ptr, const int32_t* __restrict__ strip_c,
                              uint16_t* __restrict__ lidx, const int64_t* __restrict__ lidx_ptr,
                              const int32_t* __restrict__ slice_w, uint32_t* __restrict__ pos_dl)
{
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pos) return;
  const int64_t sl = p >> 6;
  const int lane = (int)(p & 63);
  if (snode_ptr_old[sl + 1] - snode_ptr_old[sl] > 256) return;
  const uint8_t* q = q_of_u + sl * 256;
  uint8_t* su = strip_u + strip_ptr[sl] + lane * 16;
  const int steps = 16 * strip_c[sl];
  for (int j = 0; j < steps; ++j) {
    uint8_t& b = su[(int64_t)(j >> 4) * 1024 + (j & 15)];
    b = q[b];
  }
  uint16_t* li = lidx + lidx_ptr[sl] + lane;
  for (int t = 0; t < slice_w[sl]; ++t) li[64 * t] = q[li[64 * t] & 0xFFu];
  const uint32_t dl = pos_dl[p];
  pos_dl[p] = (dl & 0xFFFFu) | ((uint32_t)q[(dl >> 16) & 0xFFu] << 16);
}

__global__ void k_max_i32(int64_t n, const int32_t* __restrict__ v, unsigned long long* __restrict__ out)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) atomicMax(out, (unsigned long long)v[i]);
}

// per slice: does every lane run the same strip topology?  Uniform = one
// strip (kinds 2,2 then 0/1 only), the same length, the same shift/swap
// sequence and the same step bytes (slots) on every active row, and the same
// diagonal slot: every interior brick / face tile of a structured mesh, whose
// rows have the same sorted neighbour pattern.  Out: flag (1 = uniform), the
// swap bits (bit j = step j is a swap) and the common step bytes (32: the
// scalar slot stream of the uniform kernel; padding steps carry the diagonal
// slot).  One wave per slice.
// same[i] = 1: slice i's local-index stream (strip_u, nch[i] chunks of 1 KB)
// equals the one at rep[i] byte for byte (one 64-lane block per slice)
__global__ __launch_bounds__(64) void k_strip_same(int64_t n, const uint32_t* __restrict__ off,
                                                   const uint32_t* __restrict__ rep, const int32_t* __restrict__ nch,
                                                   const uint8_t* __restrict__ strip_u, uint8_t* __restrict__ same)
{
  const int64_t i = blockIdx.x;
  if (i >= n) return;
  const uint32_t* a = reinterpret_cast<const uint32_t*>(strip_u + (int64_t)off[i] * 1024);
  const uint32_t* b = reinterpret_cast<const uint32_t*>(strip_u + (int64_t)rep[i] * 1024);
  bool eq = true;
  for (int w = threadIdx.x; w < nch[i] * 256; w += 64) eq = eq && a[w] == b[w];
  const bool all = __all(eq);
  if (threadIdx.x == 0) same[i] = all ? 1 : 0;
}

__global__ __launch_bounds__(64) void k_strip_classify(int64_t n_slices, const int32_t* __restrict__ perm,
                                                       const uint8_t* __restrict__ strip,
                                                       const int64_t* __restrict__ strip_ptr,
                                                       const int32_t* __restrict__ strip_n,
                                                       const int64_t* __restrict__ snode_ptr,
                                                       const int32_t* __restrict__ slice_w,
                                                       const uint8_t* __restrict__ dslot, uint8_t* __restrict__ uflag,
                                                       uint64_t* __restrict__ spat, uint8_t* __restrict__ sslot)
{
  const int64_t sl = blockIdx.x;
  const int lane = threadIdx.x;
  if (sl >= n_slices) return;
  const int n = strip_n[sl];
  const uint8_t* st = strip + strip_ptr[sl] + lane * 16;
  // the uniform kernel also drops the overflow paths (> 256 slice nodes, > 16 slots).
  // Idle lanes (no row, all-padding stream: slot 0 = a zero edge) are allowed:
  // in the uniform kernel they only add zeros to their own accumulators.
  const bool idle = perm[sl * 64 + lane] < 0;
  bool ok = n >= 3 && n <= 64 && snode_ptr[sl + 1] - snode_ptr[sl] <= 256 && slice_w[sl] <= 16;
  uint64_t pat = 0;
  for (int j = 0; j < n && ok && !idle; ++j) {
    const uint32_t kind = st[(int64_t)(j >> 4) * 1024 + (j & 15)] >> 6;
    if (j < 2) ok = kind == 2;
    else if (kind > 1) ok = false;
    else pat |= (uint64_t)kind << j;
  }
  const unsigned long long act = __ballot(!idle);
  const int first = act ? __ffsll((long long)act) - 1 : 0;
  const uint64_t p0 = __shfl(pat, first);
  bool all = act != 0 && __all(ok && (idle || pat == p0));
  // slot-uniform: the same byte at every step (and the same diagonal slot)
  const uint32_t ds = dslot[sl * 64 + lane], ds0 = __shfl(ds, first);
  bool same = idle || ds == ds0;
  for (int j = 0; j < 32; ++j) {
    const uint32_t b = j < n ? st[(int64_t)(j >> 4) * 1024 + (j & 15)] : (ds | (3u << 6));
    const uint32_t b0 = __shfl(b, first);
    if (!idle && b != b0) same = false;
    if (lane == 0) sslot[sl * 32 + j] = (uint8_t)b0;
  }
  all = all && __all(same) && n <= 32;
  if (lane == 0) {
    uflag[sl] = all ? 1 : 0;
    spat[sl] = all ? p0 : 0;
  }
}

// per slice: 16-step chunks (max stream length over its lanes) and bytes
__global__ void k_strip_width(int64_t n_slices, const int32_t* __restrict__ strip_len, int32_t* __restrict__ strip_c,
                              int32_t* __restrict__ strip_n, int64_t* __restrict__ sz, int32_t* __restrict__ flags)
{
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_slices) return;
  int w = 0;
  for (int l = 0; l < 64; ++l) {
    const int v = strip_len[s * 64 + l];
    if (v < 0) atomicOr(&flags[0], 1);
    w = v > w ? v : w;
  }
  const int c = (w + 15) >> 4;
  strip_c[s] = c;
  strip_n[s] = w;
  sz[s] = (int64_t)c * 1024;
  atomicMax(&flags[1], c);
}

}  // namespace

// the owned nodes' lattice (see k_axis_keys): on success every owned node's
// layer index per axis in layer[0..2] (the sorted-coordinate order of each
// axis), the layer counts in L and true
bool lattice_coords(Ctx& ctx, const Mesh& m, int64_t n_rows, DevBuf<int32_t> layer[3], int64_t L[3])
{
  DevBuf<uint64_t> keys, keys_s;
  DevBuf<int32_t> ids, ids_s, flag;
  DevBuf<int64_t> scan;
  keys.alloc(n_rows);
  keys_s.alloc(n_rows);
  ids.alloc(n_rows);
  ids_s.alloc(n_rows);
  flag.alloc(n_rows);
  scan.alloc(n_rows + 1);
  size_t tmp_bytes = 0;
  AFEM_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, keys.p, keys_s.p, ids.p, ids_s.p, (int)n_rows, 0, 64,
                                              ctx.stream));
  DevBuf<unsigned char> tmp;
  tmp.alloc(tmp_bytes > 0 ? tmp_bytes : 1);
  DevBuf<unsigned long long> gap;
  gap.alloc(1);
  for (int a = 0; a < 3; ++a) {
    hipLaunchKernelGGL(k_axis_keys, dim3(grid_for(n_rows, 256)), dim3(256), 0, ctx.stream, n_rows, m.coords.p, a,
                       keys.p, ids.p);
    AFEM_LAUNCHED();
    AFEM_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.p, tmp_bytes, keys.p, keys_s.p, ids.p, ids_s.p, (int)n_rows, 0,
                                                64, ctx.stream));
    AFEM_HIP(hipMemsetAsync(gap.p, 0, gap.bytes(), ctx.stream));
    hipLaunchKernelGGL(k_max_gap, dim3(1024), dim3(256), 0, ctx.stream, n_rows, keys_s.p, gap.p);
    AFEM_LAUNCHED();
    unsigned long long hg = 0;
    AFEM_HIP(hipMemcpyAsync(&hg, gap.p, sizeof(hg), hipMemcpyDeviceToHost, ctx.stream));
    ctx.sync();
    double g;
    memcpy(&g, &hg, sizeof(g));
    if (!(g > 0.0)) return false;
    hipLaunchKernelGGL(k_gap_flags, dim3(grid_for(n_rows, 256)), dim3(256), 0, ctx.stream, n_rows, keys_s.p, 0.5 * g,
                       flag.p);
    AFEM_LAUNCHED();
    exclusive_scan_i32_to_i64(ctx, flag.p, scan.p, n_rows);
    L[a] = read_i64(ctx, scan.p + n_rows) + 1;
    layer[a].alloc(n_rows);
    hipLaunchKernelGGL(k_layer_scatter, dim3(grid_for(n_rows, 256)), dim3(256), 0, ctx.stream, n_rows, ids_s.p,
                       scan.p, layer[a].p);
    AFEM_LAUNCHED();
  }
  if (L[0] < 2 || L[1] < 2 || L[2] < 2 || L[0] * L[1] * L[2] != n_rows) return false;
  return true;
}

namespace {
// the brick order of the owned nodes' lattice (lattice_coords) in s.perm
// (s.n_slices, s.run, s.brick_order set) and true, or false (no lattice)
bool lattice_order(Ctx& ctx, const Mesh& m, int64_t n_rows, Structure& s)
{
  DevBuf<int32_t> layer[3];
  int64_t L[3];
  if (!lattice_coords(ctx, m, n_rows, layer, L)) return false;
  DevBuf<int32_t> lat, bad;
  lat.alloc(n_rows);
  bad.alloc(1);
  AFEM_HIP(hipMemsetAsync(lat.p, 0xFF, lat.bytes(), ctx.stream));
  AFEM_HIP(hipMemsetAsync(bad.p, 0, bad.bytes(), ctx.stream));
  hipLaunchKernelGGL(k_lattice_fill, dim3(grid_for(n_rows, 256)), dim3(256), 0, ctx.stream, n_rows, layer[0].p,
                     layer[1].p, layer[2].p, L[0], L[1], lat.p, bad.p);
  AFEM_LAUNCHED();
  int32_t hb = 0;
  AFEM_HIP(hipMemcpyAsync(&hb, bad.p, sizeof(hb), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  if (hb) return false;
  const FaceTiles F = face_tiles(L[0], L[1], L[2]);
  s.n_slices = F.start[F.nseg];
  s.perm.alloc(s.n_slices * 64);
  hipLaunchKernelGGL(k_perm_bricks_bd, dim3(grid_for(s.n_slices * 64, 256)), dim3(256), 0, ctx.stream, s.n_slices,
                     L[0], L[1], L[2], F, s.perm.p);
  AFEM_LAUNCHED();
  hipLaunchKernelGGL(k_perm_map, dim3(grid_for(s.n_slices * 64, 256)), dim3(256), 0, ctx.stream, s.n_slices * 64,
                     lat.p, s.perm.p);
  AFEM_LAUNCHED();
  ctx.sync();
  s.run = 1;
  s.brick_order = true;
  s.lattice = true;
  return true;
}
}  // namespace

int64_t node_cell_adjacency(Ctx& ctx, const Mesh& m, int64_t n_rows, DevBuf<int64_t>& nc_ptr, DevBuf<int32_t>& nc)
{
  const int nv = m.nv;
  DevBuf<int32_t> cnt;
  cnt.alloc(n_rows);
  AFEM_HIP(hipMemsetAsync(cnt.p, 0, cnt.bytes(), ctx.stream));
  const int64_t n_entries = m.n_cells * nv;
  if (n_entries) {
    hipLaunchKernelGGL(k_count_incidence, dim3(grid_for(n_entries, 256)), dim3(256), 0, ctx.stream, n_entries,
                       m.cell_node.p, n_rows, cnt.p);
    AFEM_LAUNCHED();
  }
  nc_ptr.alloc(n_rows + 1);
  exclusive_scan_i32_to_i64(ctx, cnt.p, nc_ptr.p, n_rows);
  const int64_t n_inc = read_i64(ctx, nc_ptr.p + n_rows);
  nc.alloc(n_inc > 0 ? n_inc : 1);
  AFEM_HIP(hipMemsetAsync(cnt.p, 0, cnt.bytes(), ctx.stream));
  if (n_entries) {
    hipLaunchKernelGGL(k_fill_incidence, dim3(grid_for(n_entries, 256)), dim3(256), 0, ctx.stream, m.n_cells, nv,
                       m.cell_node.p, n_rows, nc_ptr.p, cnt.p, nc.p);
    AFEM_LAUNCHED();
  }
  hipLaunchKernelGGL(k_sort_lists, dim3(grid_for(n_rows, 256)), dim3(256), 0, ctx.stream, n_rows, nc_ptr.p, nc.p);
  AFEM_LAUNCHED();
  return n_inc;
}

namespace {
void build_structure_impl(Mesh& m, Structure& s)
{
  Ctx& ctx = *m.ctx;
  ctx.set_device();
  const int64_t n_rows = m.n_own;
  const int nv = m.nv;
  s.n_rows = n_rows;
  s.n_cols = m.n_nodes;
  AFEM_REQUIRE(n_rows > 0, AFEM_ERR_ARG, "computeSparsity: mesh has no owned node");

  // 1. node -> cell adjacency of owned nodes
  DevBuf<int64_t> nc_ptr;
  DevBuf<int32_t> nc;
  s.n_incidences = node_cell_adjacency(ctx, m, n_rows, nc_ptr, nc);

  // 2. rows = sorted unique union of incident cells' nodes
  DevBuf<int32_t> row_len;
  row_len.alloc(n_rows);
  hipLaunchKernelGGL(k_row_union<false>, dim3(grid_for(n_rows, kUnionThreads)), dim3(kUnionThreads), 0, ctx.stream,
                     n_rows, nv, m.cell_node.p, nc_ptr.p, nc.p, row_len.p, nullptr, nullptr, nullptr);
  AFEM_LAUNCHED();
  DevBuf<int32_t> flags;
  flags.alloc(2);
  AFEM_HIP(hipMemsetAsync(flags.p, 0, flags.bytes(), ctx.stream));
  hipLaunchKernelGGL(k_check_len, dim3(grid_for(n_rows, 256)), dim3(256), 0, ctx.stream, n_rows, row_len.p, flags.p);
  AFEM_LAUNCHED();
  int32_t hflags[2];
  AFEM_HIP(hipMemcpyAsync(hflags, flags.p, sizeof(hflags), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  AFEM_REQUIRE(hflags[0] == 0, AFEM_ERR_LIMIT,
               "computeSparsity: a row has more than 255 non-zero blocks (node degree limit of the 8-bit slot table)");
  s.max_row_len = hflags[1];
  s.row_ptr.alloc(n_rows + 1);
  exclusive_scan_i32_to_i64(ctx, row_len.p, s.row_ptr.p, n_rows);
  s.nnz = read_i64(ctx, s.row_ptr.p + n_rows);
  s.cols.alloc(s.nnz + 4);  // tail padding: the assembly stages columns with 16-B loads
  AFEM_HIP(hipMemsetAsync(s.cols.p + s.nnz, 0, 4 * sizeof(int32_t), ctx.stream));
  s.diag_pos.alloc(n_rows);
  hipLaunchKernelGGL(k_row_union<true>, dim3(grid_for(n_rows, kUnionThreads)), dim3(kUnionThreads), 0, ctx.stream,
                     n_rows, nv, m.cell_node.p, nc_ptr.p, nc.p, nullptr, s.row_ptr.p, s.cols.p, s.diag_pos.p);
  AFEM_LAUNCHED();

  // 3. processing order (slices of 64 rows)
  const StructuredInfo& st = m.st;
  if (st.valid && (st.dim == 3 || st.dim == 2)) {
    const int64_t ax = st.lx > 0 ? st.lx : st.n + 1;
    const int64_t own_layers = st.k1 - st.k0;
    const int64_t ay = st.dim == 3 ? (st.ly > 0 ? st.ly : (int64_t)st.n + 1) : own_layers;
    const int64_t az = st.dim == 3 ? own_layers : 1;
    AFEM_REQUIRE(ax * ay * az == n_rows, AFEM_ERR_STATE, "structured mesh: owned node box does not match n_own");
    const int bx = st.dim == 3 ? 4 : 8, bz = st.dim == 3 ? 4 : 1;
    // AFEM_BRICKS=plain: the plain 4x4x4 brick grid over the whole box (diagnostic)
    const char* be = variant("AFEM_BRICKS");
    const bool boundary_aware = st.dim == 3 && !(be && std::string(be) == "plain");
    if (boundary_aware) {
      const FaceTiles F = face_tiles(ax, ay, az);
      s.n_slices = F.start[F.nseg];
      s.perm.alloc(s.n_slices * 64);
      hipLaunchKernelGGL(k_perm_bricks_bd, dim3(grid_for(s.n_slices * 64, 256)), dim3(256), 0, ctx.stream,
                         s.n_slices, ax, ay, az, F, s.perm.p);
      AFEM_LAUNCHED();
      DevBuf<unsigned long long> cnt;
      cnt.alloc(1);
      AFEM_HIP(hipMemsetAsync(cnt.p, 0, cnt.bytes(), ctx.stream));
      hipLaunchKernelGGL(k_count_valid, dim3(grid_for(s.n_slices * 64, 256)), dim3(256), 0, ctx.stream,
                         s.n_slices * 64, s.perm.p, cnt.p);
      AFEM_LAUNCHED();
      unsigned long long hc = 0;
      AFEM_HIP(hipMemcpyAsync(&hc, cnt.p, sizeof(hc), hipMemcpyDeviceToHost, ctx.stream));
      ctx.sync();
      AFEM_REQUIRE((int64_t)hc == n_rows, AFEM_ERR_STATE, "boundary-aware brick order does not cover the owned nodes");
      s.run = 1;  // face tiles of the i planes do not hold consecutive rows
    }
    else {
      s.n_slices = ((ax + bx - 1) / bx) * ((ay + bx - 1) / bx) * ((az + bz - 1) / bz);
      s.perm.alloc(s.n_slices * 64);
      hipLaunchKernelGGL(k_perm_bricks, dim3(grid_for(s.n_slices * 64, 256)), dim3(256), 0, ctx.stream, s.n_slices,
                         st.dim, ax, ay, az, s.perm.p);
      AFEM_LAUNCHED();
      s.run = st.dim == 3 ? 4 : 8;
    }
    s.brick_order = true;
  }
  else if (!(nv == 4 && m.dim == 3 && n_rows >= 8 && !variant("AFEM_ORDER") && lattice_order(ctx, m, n_rows, s))) {
    s.n_slices = (n_rows + 63) / 64;
    s.perm.alloc(s.n_slices * 64);
    // AFEM_ORDER=node: the caller's node order; =morton: Morton curve; =hilbert:
    // the Hilbert curve even for a lattice (diagnostics)
    const char* oe = variant("AFEM_ORDER");
    const bool node_order = (oe && std::string(oe) == "node") || n_rows < 2;
    if (node_order) {
      hipLaunchKernelGGL(k_perm_identity, dim3(grid_for(s.n_slices * 64, 256)), dim3(256), 0, ctx.stream,
                         s.n_slices * 64, n_rows, s.perm.p);
      AFEM_LAUNCHED();
      s.run = 64;
    }
    else {
      DevBuf<unsigned long long> box;
      box.alloc(6);
      const unsigned long long init[6] = { ~0ull, ~0ull, ~0ull, 0ull, 0ull, 0ull };
      AFEM_HIP(hipMemcpyAsync(box.p, init, sizeof(init), hipMemcpyHostToDevice, ctx.stream));
      hipLaunchKernelGGL(k_bbox, dim3(1024), dim3(256), 0, ctx.stream, n_rows, m.coords.p, box.p);
      AFEM_LAUNCHED();
      DevBuf<uint64_t> keys, keys_out;
      DevBuf<int32_t> ids, ids_out;
      keys.alloc(n_rows);
      keys_out.alloc(n_rows);
      ids.alloc(n_rows);
      ids_out.alloc(n_rows);
      if (oe && std::string(oe) == "morton")
        hipLaunchKernelGGL(k_curve_keys<false>, dim3(grid_for(n_rows, 256)), dim3(256), 0, ctx.stream, n_rows,
                           m.coords.p, box.p, keys.p, ids.p);
      else
        hipLaunchKernelGGL(k_curve_keys<true>, dim3(grid_for(n_rows, 256)), dim3(256), 0, ctx.stream, n_rows,
                           m.coords.p, box.p, keys.p, ids.p);
      AFEM_LAUNCHED();
      size_t tmp_bytes = 0;
      AFEM_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, keys.p, keys_out.p, ids.p, ids_out.p,
                                                  (int)n_rows, 0, 64, ctx.stream));
      DevBuf<unsigned char> tmp;
      tmp.alloc(tmp_bytes > 0 ? tmp_bytes : 1);
      AFEM_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.p, tmp_bytes, keys.p, keys_out.p, ids.p, ids_out.p,
                                                  (int)n_rows, 0, 64, ctx.stream));
      hipLaunchKernelGGL(k_perm_from_sorted, dim3(grid_for(s.n_slices * 64, 256)), dim3(256), 0, ctx.stream,
                         s.n_slices * 64, n_rows, ids_out.p, s.perm.p);
      AFEM_LAUNCHED();
      ctx.sync();
      s.run = 1;  // a slice's rows are spatial neighbours, not consecutive rows
    }
    s.brick_order = false;
  }
  const int64_t n_pos = s.n_slices * 64;

  // 4. sliced-ELL row-local incidence table in processing order
  s.inc_slice_k.alloc(s.n_slices);
  DevBuf<int64_t> slice_sz;
  slice_sz.alloc(s.n_slices);
  hipLaunchKernelGGL(k_slice_width, dim3(grid_for(s.n_slices, 256)), dim3(256), 0, ctx.stream, s.n_slices, s.perm.p,
                     nc_ptr.p, s.inc_slice_k.p, slice_sz.p);
  AFEM_LAUNCHED();
  s.inc_slice_ptr.alloc(s.n_slices + 1);
  exclusive_scan_i64(ctx, slice_sz.p, s.inc_slice_ptr.p, s.n_slices);
  const int64_t inc_total = read_i64(ctx, s.inc_slice_ptr.p + s.n_slices);
  s.inc.alloc(inc_total + 256);
  s.inc_pad_off = inc_total;
  AFEM_HIP(hipMemsetAsync(s.inc.p + inc_total, 0xFF, 256 * sizeof(uint32_t), ctx.stream));
  hipLaunchKernelGGL(k_fill_inc, dim3(grid_for(n_pos, 256)), dim3(256), 0, ctx.stream, n_pos, nv, s.perm.p,
                     m.cell_node.p, nc_ptr.p, nc.p, s.row_ptr.p, s.cols.p, s.inc_slice_ptr.p, s.inc_slice_k.p, s.inc.p);
  AFEM_LAUNCHED();

  // 5. slice node lists + local column indices
  int m_cap = 64;
  while (m_cap < 64 * s.max_row_len) m_cap <<= 1;
  s.slice_w.alloc(s.n_slices);
  DevBuf<int64_t> slice_nu;
  slice_nu.alloc(s.n_slices);
  hipLaunchKernelGGL(k_slice_nodes<false>, dim3((unsigned)s.n_slices), dim3(64), (size_t)m_cap * 4, ctx.stream,
                     s.perm.p, s.row_ptr.p, s.cols.p, s.slice_w.p, slice_nu.p, nullptr, nullptr, nullptr, nullptr);
  AFEM_LAUNCHED();
  s.snode_ptr.alloc(s.n_slices + 1);
  exclusive_scan_i64(ctx, slice_nu.p, s.snode_ptr.p, s.n_slices);
  const int64_t n_snode = read_i64(ctx, s.snode_ptr.p + s.n_slices);
  hipLaunchKernelGGL(k_times64, dim3(grid_for(s.n_slices, 256)), dim3(256), 0, ctx.stream, s.n_slices, s.slice_w.p,
                     slice_sz.p);
  AFEM_LAUNCHED();
  s.lidx_ptr.alloc(s.n_slices + 1);
  exclusive_scan_i64(ctx, slice_sz.p, s.lidx_ptr.p, s.n_slices);
  const int64_t n_lidx = read_i64(ctx, s.lidx_ptr.p + s.n_slices);
  s.snode.alloc(n_snode > 0 ? n_snode : 1);
  s.lidx.alloc(n_lidx + 8);  // tail: the assembly stages the table with 16-B loads
  hipLaunchKernelGGL(k_slice_nodes<true>, dim3((unsigned)s.n_slices), dim3(64), (size_t)m_cap * 4, ctx.stream,
                     s.perm.p, s.row_ptr.p, s.cols.p, nullptr, nullptr, s.snode_ptr.p, s.snode.p, s.lidx_ptr.p,
                     s.lidx.p);
  AFEM_LAUNCHED();
  {
    DevBuf<unsigned long long> mx;
    mx.alloc(4);
    AFEM_HIP(hipMemsetAsync(mx.p, 0, mx.bytes(), ctx.stream));
    hipLaunchKernelGGL(k_slice_max, dim3(grid_for(s.n_slices, 256)), dim3(256), 0, ctx.stream, s.n_slices, s.perm.p,
                       s.row_ptr.p, s.slice_w.p, slice_nu.p, s.inc_slice_k.p, mx.p);
    AFEM_LAUNCHED();
    unsigned long long hm[4] = { 0, 0, 0, 0 };
    AFEM_HIP(hipMemcpyAsync(hm, mx.p, sizeof(hm), hipMemcpyDeviceToHost, ctx.stream));
    ctx.sync();
    s.max_wave_seg = (int64_t)hm[0];
    s.max_slice_w = (int)hm[1];
    s.max_slice_nodes = (int)hm[2];
    s.max_slice_k = (int)hm[3];
  }

  // 6. row strips (the scalar assembly's cell order and node stream)
  {
    DevBuf<int32_t> slen;
    slen.alloc(n_pos);
    hipLaunchKernelGGL(k_strip_rows<false>, dim3(grid_for(n_pos, 64)), dim3(64), 0, ctx.stream, n_pos, nv, s.perm.p,
                       m.cell_node.p, nc_ptr.p, nc.p, s.row_ptr.p, s.cols.p, slen.p, nullptr, nullptr, nullptr,
                       nullptr);
    AFEM_LAUNCHED();
    s.strip_c.alloc(s.n_slices);
    s.strip_n.alloc(s.n_slices);
    DevBuf<int64_t> ssz;
    ssz.alloc(s.n_slices);
    DevBuf<int32_t> sflags;
    sflags.alloc(2);
    AFEM_HIP(hipMemsetAsync(sflags.p, 0, sflags.bytes(), ctx.stream));
    hipLaunchKernelGGL(k_strip_width, dim3(grid_for(s.n_slices, 256)), dim3(256), 0, ctx.stream, s.n_slices, slen.p,
                       s.strip_c.p, s.strip_n.p, ssz.p, sflags.p);
    AFEM_LAUNCHED();
    int32_t hf[2] = { 0, 0 };
    AFEM_HIP(hipMemcpyAsync(hf, sflags.p, sizeof(hf), hipMemcpyDeviceToHost, ctx.stream));
    ctx.sync();
    s.strip_ok = hf[0] == 0;
    s.max_strip_c = hf[1];
    if (s.strip_ok) {
      s.strip_ptr.alloc(s.n_slices + 1);
      exclusive_scan_i64(ctx, ssz.p, s.strip_ptr.p, s.n_slices);
      const int64_t nbytes = read_i64(ctx, s.strip_ptr.p + s.n_slices);
      s.strip.alloc(nbytes + 1024);
      s.dslot.alloc(n_pos);
      hipLaunchKernelGGL(k_strip_rows<true>, dim3(grid_for(n_pos, 64)), dim3(64), 0, ctx.stream, n_pos, nv,
                         s.perm.p, m.cell_node.p, nc_ptr.p, nc.p, s.row_ptr.p, s.cols.p, nullptr, s.strip_ptr.p,
                         s.strip_c.p, s.strip.p, s.dslot.p);
      AFEM_LAUNCHED();
      // per-position row data of the strip assembly
      s.pos_rb.alloc(n_pos);
      s.pos_dl.alloc(n_pos);
      hipLaunchKernelGGL(k_pos_rows, dim3(grid_for(n_pos, 256)), dim3(256), 0, ctx.stream, n_pos, s.perm.p,
                         s.row_ptr.p, s.dslot.p, s.lidx_ptr.p, s.lidx.p, s.pos_rb.p, s.pos_dl.p);
      AFEM_LAUNCHED();
      s.strip_u.alloc(s.strip.n);
      hipLaunchKernelGGL(k_strip_local, dim3(grid_for(n_pos, 256)), dim3(256), 0, ctx.stream, n_pos, s.strip.p,
                         s.strip_ptr.p, s.strip_c.p, s.lidx_ptr.p, s.lidx.p, s.strip_u.p);
      AFEM_LAUNCHED();
      // uniform / mixed slice lists (tets; triangles use the general path)
      DevBuf<uint8_t> uflag;
      uflag.alloc(s.n_slices);
      s.spat.alloc(s.n_slices);
      DevBuf<uint8_t> sslot;
      sslot.alloc(s.n_slices * 32);
      hipLaunchKernelGGL(k_strip_classify, dim3((unsigned)s.n_slices), dim3(64), 0, ctx.stream, s.n_slices, s.perm.p,
                         s.strip.p, s.strip_ptr.p, s.strip_n.p, s.snode_ptr.p, s.slice_w.p, s.dslot.p, uflag.p,
                         s.spat.p, sslot.p);
      AFEM_LAUNCHED();
      // LDS-bank-aware node placement of the uniform slices (AFEM_BANK_PLACE=0: sorted order, diagnostic)
      const char* bpe = variant("AFEM_BANK_PLACE");
      if (!(bpe && atoi(bpe) == 0) && nv == 4) {
        DevBuf<uint8_t> q_of_u;
        q_of_u.alloc(s.n_slices * 256);
        DevBuf<int32_t> nu_new;
        nu_new.alloc(s.n_slices);
        // positions < maxq: 232 keeps the uniform instance's LDS image at 13.3 KB per wave
        // (12 waves per CU with 15 slots); classes c < 8 get 8 positions, the others 7
        const char* bpm = variant("AFEM_BANK_PLACE_MAX");
        const int maxq = bpm ? std::max(64, std::min(256, atoi(bpm))) : 232;
        // general slices too with AFEM_BANK_PLACE_GENERAL=1 (a greedy colouring;
        // measured on the refined L-shape: SQ_LDS_BANK_CONFLICT -4 %, kernel +2 %
        // (1.407 vs 1.380 ms, r04g) -- their conflicts are not the coordinate reads)
        const char* bge = variant("AFEM_BANK_PLACE_GENERAL");
        const int general = (bge && atoi(bge) == 1) ? 1 : 0;
        hipLaunchKernelGGL(k_bank_place, dim3((unsigned)s.n_slices), dim3(64), 0, ctx.stream, s.n_slices, uflag.p,
                           s.perm.p, s.snode_ptr.p, s.strip_u.p, s.strip_ptr.p, s.strip_n.p, s.pos_dl.p, q_of_u.p,
                           nu_new.p, maxq, general);
        AFEM_LAUNCHED();
        DevBuf<int64_t> ptr_new;
        ptr_new.alloc(s.n_slices + 1);
        exclusive_scan_i32_to_i64(ctx, nu_new.p, ptr_new.p, s.n_slices);
        const int64_t n_new = read_i64(ctx, ptr_new.p + s.n_slices);
        DevBuf<int32_t> snode_new;
        snode_new.alloc(n_new > 0 ? n_new : 1);
        hipLaunchKernelGGL(k_snode_place, dim3((unsigned)s.n_slices), dim3(64), 0, ctx.stream, s.n_slices,
                           s.snode_ptr.p, s.snode.p, ptr_new.p, snode_new.p, q_of_u.p);
        AFEM_LAUNCHED();
        hipLaunchKernelGGL(k_local_place, dim3(grid_for(n_pos, 256)), dim3(256), 0, ctx.stream, n_pos, s.snode_ptr.p,
                           q_of_u.p, s.strip_u.p, s.strip_ptr.p, s.strip_c.p, s.lidx.p, s.lidx_ptr.p, s.slice_w.p,
                           s.pos_dl.p);
        AFEM_LAUNCHED();
        ctx.sync();
        s.snode = std::move(snode_new);
        s.snode_ptr = std::move(ptr_new);
        DevBuf<unsigned long long> mx;
        mx.alloc(1);
        AFEM_HIP(hipMemsetAsync(mx.p, 0, mx.bytes(), ctx.stream));
        hipLaunchKernelGGL(k_max_i32, dim3(grid_for(s.n_slices, 256)), dim3(256), 0, ctx.stream, s.n_slices, nu_new.p,
                           mx.p);
        AFEM_LAUNCHED();
        unsigned long long hm = 0;
        AFEM_HIP(hipMemcpyAsync(&hm, mx.p, sizeof(hm), hipMemcpyDeviceToHost, ctx.stream));
        ctx.sync();
        s.max_slice_nodes = (int)hm;
      }
      const size_t ns = (size_t)s.n_slices;
      std::vector<uint8_t> hu(ns);
      std::vector<int32_t> hw(ns), hn(ns);
      std::vector<int64_t> hl(ns + 1), hs(ns + 1), hsn(ns + 1);
      std::vector<uint64_t> hp(ns);
      std::vector<uint8_t> hslot(ns * 32);
      AFEM_HIP(hipMemcpyAsync(hslot.data(), sslot.p, ns * 32, hipMemcpyDeviceToHost, ctx.stream));
      AFEM_HIP(hipMemcpyAsync(hu.data(), uflag.p, ns, hipMemcpyDeviceToHost, ctx.stream));
      AFEM_HIP(hipMemcpyAsync(hw.data(), s.slice_w.p, ns * 4, hipMemcpyDeviceToHost, ctx.stream));
      AFEM_HIP(hipMemcpyAsync(hn.data(), s.strip_n.p, ns * 4, hipMemcpyDeviceToHost, ctx.stream));
      AFEM_HIP(hipMemcpyAsync(hl.data(), s.lidx_ptr.p, (ns + 1) * 8, hipMemcpyDeviceToHost, ctx.stream));
      AFEM_HIP(hipMemcpyAsync(hs.data(), s.strip_ptr.p, (ns + 1) * 8, hipMemcpyDeviceToHost, ctx.stream));
      AFEM_HIP(hipMemcpyAsync(hsn.data(), s.snode_ptr.p, (ns + 1) * 8, hipMemcpyDeviceToHost, ctx.stream));
      AFEM_HIP(hipMemcpyAsync(hp.data(), s.spat.p, ns * 8, hipMemcpyDeviceToHost, ctx.stream));
      ctx.sync();
      s.rec_ok = hl[ns] < (int64_t(1) << 32) && hs[ns] / 1024 < (int64_t(1) << 32) && hsn[ns] < (int64_t(1) << 32);
      std::vector<SliceRec> ru, rm, ra;
      std::vector<uint8_t> su;  // the uniform list's slot streams, in list order
      for (size_t i = 0; i < ns && s.rec_ok; ++i) {
        SliceRec r{};
        r.sl = (uint32_t)i;
        r.lidx_off = (uint32_t)hl[i];
        r.strip_off = (uint32_t)(hs[i] / 1024);
        r.snode_off = (uint32_t)hsn[i];
        const int64_t nu = hsn[i + 1] - hsn[i];
        if (nu > 65535 || hw[i] > 255 || hn[i] > 255) s.rec_ok = false;
        r.meta = (uint32_t)nu | (uint32_t)hw[i] << 16 | (uint32_t)hn[i] << 24;
        r.pat = hp[i];
        ra.push_back(r);
        if (hu[i] && nv == 4) {
          ru.push_back(r);
          su.insert(su.end(), hslot.begin() + 32 * i, hslot.begin() + 32 * (i + 1));
        }
        else {
          rm.push_back(r);
        }
      }
      s.n_uni = (int64_t)ru.size();
      s.n_mix = (int64_t)rm.size();
      constexpr int kSmallSliceNodes = 352;
      auto small_slice = [&](const SliceRec& r) {
        return (int)((r.meta >> 16) & 0xFFu) <= 16 && (int)(r.meta >> 24) <= 32 &&
               (int)(r.meta & 0xFFFFu) <= kSmallSliceNodes;
      };
      std::vector<SliceRec> ms_h;  // the compact general list, host copy (the stencil split may extend it)
      // upload of the compact list, its slices of <= 256 nodes first (stable: each
      // part keeps the processing order), n_msl of them
      auto upload_ms = [&](std::vector<SliceRec>& h) {
        std::stable_partition(h.begin(), h.end(), [](const SliceRec& r) { return (r.meta & 0xFFFFu) <= 256; });
        s.n_msl = 0;
        s.msl_nodes = 0;
        for (const SliceRec& r : h)
          if ((r.meta & 0xFFFFu) <= 256) {
            ++s.n_msl;
            s.msl_nodes = std::max(s.msl_nodes, (int)(r.meta & 0xFFFFu));
          }
        s.rec_ms.alloc(h.empty() ? 1 : h.size());
        if (!h.empty())
          AFEM_HIP(hipMemcpyAsync(s.rec_ms.p, h.data(), h.size() * sizeof(SliceRec), hipMemcpyHostToDevice, ctx.stream));
        ctx.sync();  // h may change before the copy ran
      };
      {
        // general-instance slices: the compact ones (<= 16 slots, <= 32 steps,
        // <= 352 nodes: 90 % of a Hilbert-ordered unstructured mesh) in their
        // own list, so the big ones do not size the LDS tile of all
        std::vector<SliceRec> ms, mb;
        s.ms_nodes = s.mb_nodes = s.mb_w = 0;
        for (const SliceRec& r : rm) {
          const int nu = (int)(r.meta & 0xFFFFu), w = (int)((r.meta >> 16) & 0xFFu);
          if (small_slice(r)) {
            ms.push_back(r);
            s.ms_nodes = std::max(s.ms_nodes, nu);
          }
          else {
            mb.push_back(r);
            s.mb_nodes = std::max(s.mb_nodes, nu);
            s.mb_w = std::max(s.mb_w, w);
          }
        }
        s.u_nodes = s.u_w = 0;
        for (const SliceRec& r : ru) {
          s.u_nodes = std::max(s.u_nodes, (int)(r.meta & 0xFFFFu));
          s.u_w = std::max(s.u_w, (int)((r.meta >> 16) & 0xFFu));
        }
        s.n_ms = (int64_t)ms.size();
        s.n_mb = (int64_t)mb.size();
        auto up = [&](DevBuf<SliceRec>& d, const std::vector<SliceRec>& h) {
          d.alloc(h.empty() ? 1 : h.size());
          if (!h.empty())
            AFEM_HIP(hipMemcpyAsync(d.p, h.data(), h.size() * sizeof(SliceRec), hipMemcpyHostToDevice, ctx.stream));
        };
        ms_h = std::move(ms);
        upload_ms(ms_h);
        up(s.rec_mb, mb);
      }
      auto upload = [&](DevBuf<SliceRec>& d, const std::vector<SliceRec>& h) {
        d.alloc(h.empty() ? 1 : h.size());
        if (!h.empty())
          AFEM_HIP(hipMemcpyAsync(d.p, h.data(), h.size() * sizeof(SliceRec), hipMemcpyHostToDevice, ctx.stream));
      };
      upload(s.rec_u, ru);
      s.uslot.alloc(su.empty() ? 32 : su.size());
      if (!su.empty()) AFEM_HIP(hipMemcpyAsync(s.uslot.p, su.data(), su.size(), hipMemcpyHostToDevice, ctx.stream));
      {
        // stencil split of the uniform list (scalar assembly): the slices of a
        // compiled-in signature run k_assemble_stencil (one kernel for all
        // signatures, SliceRec::sig), the other uniform slices the uniform
        // instance (rec_ur with their slot streams)
        std::vector<int> sid(ru.size());
        std::map<int, int64_t> cnt;
        for (size_t i = 0; i < ru.size(); ++i) {
          const SliceRec& r = ru[i];
          sid[i] = stencil_match(r.pat, (int)(r.meta >> 24), (int)((r.meta >> 16) & 0xFFu), su.data() + 32 * i);
          if (sid[i] >= 0) ++cnt[sid[i]];
        }
        int best = -1;
        for (const auto& kv : cnt)
          if (best < 0 || kv.second > cnt[best]) best = kv.first;
        std::vector<SliceRec> rk, rur, rk0, ru1;
        std::vector<uint8_t> sur, su1;
        s.k_nodes = s.ur_nodes = s.ur_w = 0;
        for (size_t i = 0; i < ru.size(); ++i) {
          const SliceRec& r = ru[i];
          if (sid[i] >= 0) {
            rk.push_back(r);
            rk.back().sig = (uint32_t)sid[i];
            s.k_nodes = std::max(s.k_nodes, (int)(r.meta & 0xFFFFu));
          }
          else {
            rur.push_back(r);
            sur.insert(sur.end(), su.begin() + 32 * i, su.begin() + 32 * (i + 1));
            s.ur_nodes = std::max(s.ur_nodes, (int)(r.meta & 0xFFFFu));
            s.ur_w = std::max(s.ur_w, (int)((r.meta >> 16) & 0xFFu));
          }
        }
        // a few uniform slices without a compiled-in signature beside the stencil
        // slices (a box's edge runs and corners, boundary_aware order) join the
        // compact general list: one small launch before the stencil kernel
        // instead of two (AFEM_ASSEMBLY_FOLD=0 keeps them on the uniform instance)
        const char* fe = variant("AFEM_ASSEMBLY_FOLD");
        if (!(fe && atoi(fe) == 0) && !rk.empty() && !rur.empty() && rur.size() * 256 <= rk.size() &&
            std::all_of(rur.begin(), rur.end(), small_slice)) {
          for (const SliceRec& r : rur) {
            ms_h.push_back(r);
            s.ms_nodes = std::max(s.ms_nodes, (int)(r.meta & 0xFFFFu));
          }
          s.n_ms = (int64_t)ms_h.size();
          upload_ms(ms_h);
          rur.clear();
          sur.clear();
          s.ur_nodes = s.ur_w = 0;
        }
        s.sig_k = best;
        s.n_k = (int64_t)rk.size();
        s.n_ur = (int64_t)rur.size();
        // Interior bricks of one signature have byte-identical local-index streams
        // (same strip, same node-list layout and bank placement): those slices read
        // the signature's first copy (2 KB, L2-resident) instead of their own --
        // 32 B per row less HBM traffic.  Verified byte for byte (k_strip_same);
        // AFEM_STRIP_SHARE=0 keeps every slice on its own stream.
        s.n_strip_shared = 0;
        const char* sse = variant("AFEM_STRIP_SHARE");
        if (!rk.empty() && !(sse && atoi(sse) == 0)) {
          const size_t nk = rk.size();
          std::map<uint32_t, uint32_t> first;  // signature -> strip_off of its first slice
          std::vector<uint32_t> ho(nk), hr(nk);
          std::vector<int32_t> hc(nk);
          for (size_t i = 0; i < nk; ++i) {
            first.emplace(rk[i].sig, rk[i].strip_off);
            ho[i] = rk[i].strip_off;
            hr[i] = first[rk[i].sig];
            hc[i] = (int32_t)((hs[rk[i].sl + 1] - hs[rk[i].sl]) / 1024);
          }
          DevBuf<uint32_t> doff, drep;
          DevBuf<int32_t> dnch;
          DevBuf<uint8_t> dsame;
          doff.alloc(nk);
          drep.alloc(nk);
          dnch.alloc(nk);
          dsame.alloc(nk);
          AFEM_HIP(hipMemcpyAsync(doff.p, ho.data(), nk * 4, hipMemcpyHostToDevice, ctx.stream));
          AFEM_HIP(hipMemcpyAsync(drep.p, hr.data(), nk * 4, hipMemcpyHostToDevice, ctx.stream));
          AFEM_HIP(hipMemcpyAsync(dnch.p, hc.data(), nk * 4, hipMemcpyHostToDevice, ctx.stream));
          hipLaunchKernelGGL(k_strip_same, dim3((unsigned)nk), dim3(64), 0, ctx.stream, (int64_t)nk, doff.p, drep.p,
                             dnch.p, s.strip_u.p, dsame.p);
          AFEM_LAUNCHED();
          std::vector<uint8_t> hsame(nk);
          AFEM_HIP(hipMemcpyAsync(hsame.data(), dsame.p, nk, hipMemcpyDeviceToHost, ctx.stream));
          ctx.sync();
          for (size_t i = 0; i < nk; ++i)
            if (hsame[i] && hr[i] != ho[i]) {
              rk[i].strip_off = hr[i];
              ++s.n_strip_shared;
            }
        }
        upload(s.rec_k, rk);
        upload(s.rec_ur, rur);
        for (size_t i = 0; i < ru.size(); ++i) {
          if (sid[i] == 0) {
            rk0.push_back(ru[i]);  // (block-3 keeps its own streams: sharing measured 1.6 % slower on C3)
          }
          else {
            ru1.push_back(ru[i]);
            su1.insert(su1.end(), su.begin() + 32 * i, su.begin() + 32 * (i + 1));
          }
        }
        s.n_k0 = (int64_t)rk0.size();
        s.n_u1 = (int64_t)ru1.size();
        upload(s.rec_k0, rk0);
        upload(s.rec_u1, ru1);
        s.u1slot.alloc(su1.empty() ? 32 : su1.size());
        if (!su1.empty())
          AFEM_HIP(hipMemcpyAsync(s.u1slot.p, su1.data(), su1.size(), hipMemcpyHostToDevice, ctx.stream));
        s.urslot.alloc(sur.empty() ? 32 : sur.size());
        if (!sur.empty())
          AFEM_HIP(hipMemcpyAsync(s.urslot.p, sur.data(), sur.size(), hipMemcpyHostToDevice, ctx.stream));
      }
      upload(s.rec_m, rm);
      upload(s.rec_all, ra);
      if (variant("AFEM_DEBUG_SLICES")) {  // diagnostic: slice node counts and widths
        std::vector<int64_t> nus(ns);
        for (size_t i = 0; i < ns; ++i) nus[i] = hsn[i + 1] - hsn[i];
        std::sort(nus.begin(), nus.end());
        std::vector<int32_t> ws(hw.begin(), hw.end());
        std::sort(ws.begin(), ws.end());
        auto q = [&](const auto& v, double f) { return (long long)v[(size_t)(f * (double)(v.size() - 1))]; };
        fprintf(stderr, "afem slices %zu nodes p50 %lld p90 %lld p99 %lld max %lld | width p50 %lld p90 %lld max %lld\n",
                ns, q(nus, 0.5), q(nus, 0.9), q(nus, 0.99), q(nus, 1.0), q(ws, 0.5), q(ws, 0.9), q(ws, 1.0));
      }
      if (variant("AFEM_DEBUG_PATTERNS")) {  // diagnostic: strip patterns of the uniform slices
        std::map<std::pair<uint64_t, int>, int64_t> h;
        std::map<std::string, int64_t> hs2;  // pattern + steps + slot stream
        for (size_t i = 0; i < ru.size(); ++i) {
          const SliceRec& r = ru[i];
          ++h[{ r.pat, (int)(r.meta >> 24) }];
          char b[32];
          snprintf(b, sizeof(b), "%016llx/%d/w%d/", (unsigned long long)r.pat, (int)(r.meta >> 24),
                   (int)((r.meta >> 16) & 0xFFu));
          std::string k(b);
          for (int t = 0; t < 32; ++t) {
            snprintf(b, sizeof(b), "%02x", su[32 * i + t]);
            k += b;
          }
          ++hs2[k];
        }
        for (auto& kv : h)
          fprintf(stderr, "afem pattern 0x%016llx steps %d slices %lld\n", (unsigned long long)kv.first.first,
                  kv.first.second, (long long)kv.second);
        std::vector<std::pair<int64_t, std::string>> top;
        for (auto& kv : hs2) top.push_back({ kv.second, kv.first });
        std::sort(top.rbegin(), top.rend());
        fprintf(stderr, "afem pattern+slots: %zu distinct\n", top.size());
        for (size_t i = 0; i < top.size() && i < 48; ++i)
          fprintf(stderr, "afem  %lld  %s\n", (long long)top[i].first, top[i].second.c_str());
      }
      ctx.sync();
    }
    else {
      s.strip_c.reset();
      s.strip_n.reset();
    }
  }
  ctx.sync();
}

// ---- canonical lattice structures.  A mesh handed over as arrays whose owned
// nodes sit on a lattice gets the brick order (lattice_order), but in a
// non-generator numbering each row's columns -- sorted by node id -- come in a
// different order from row to row, so no slice is uniform and no compiled-in
// strip signature matches.  Relabeling the nodes by their lattice index (x +
// Lx (y + Ly z): the generator's numbering) and ordering the cells by (lower
// cube corner, Kuhn type: the generator's cell order) reproduces the
// generator's structure; its slices, strips and node lists are built there and
// keep working in the caller's numbering through two maps: the nodes (perm,
// snode: lattice index -> node id) and each row's slots (cperm: canonical slot
// -> position in the row's id-sorted columns, applied by the kernels' stores).
__global__ void k_lat_ids(int64_t n, const int32_t* __restrict__ lx, const int32_t* __restrict__ ly,
                          const int32_t* __restrict__ lz, int64_t L0, int64_t L1, int32_t* __restrict__ lat,
                          int32_t* __restrict__ inv)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t id = lx[i] + L0 * (ly[i] + L1 * (int64_t)lz[i]);
  lat[i] = (int32_t)id;
  inv[id] = (int32_t)i;
}

// key of a cell: lattice index of its lower cube corner, then the Kuhn type of
// its vertex path (v1 - v0 = e_a0, v2 - v1 = e_a1: mesh.hip c_kuhn's order), 7
// for any other shape
__global__ void k_cell_keys(int64_t nc, const int32_t* __restrict__ cn, const int32_t* __restrict__ lx,
                            const int32_t* __restrict__ ly, const int32_t* __restrict__ lz, int64_t L0, int64_t L1,
                            unsigned long long* __restrict__ keys, int32_t* __restrict__ ids)
{
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nc) return;
  int x[4], y[4], z[4];
  int mx = 1 << 30, my = 1 << 30, mz = 1 << 30;
  for (int a = 0; a < 4; ++a) {
    const int32_t v = cn[4 * c + a];
    x[a] = lx[v];
    y[a] = ly[v];
    z[a] = lz[v];
    mx = min(mx, x[a]);
    my = min(my, y[a]);
    mz = min(mz, z[a]);
  }
  // vertices by lattice index (a Kuhn path climbs it at every step): the type
  // does not depend on the cell's vertex order
  auto lid = [&](int a) { return (int64_t)x[a] + L0 * ((int64_t)y[a] + L1 * (int64_t)z[a]); };
  for (int i = 1; i < 4; ++i)
    for (int j = i; j > 0 && lid(j) < lid(j - 1); --j) {
      const int tx = x[j], ty = y[j], tz = z[j];
      x[j] = x[j - 1];
      y[j] = y[j - 1];
      z[j] = z[j - 1];
      x[j - 1] = tx;
      y[j - 1] = ty;
      z[j - 1] = tz;
    }
  auto axis = [&](int a, int b) -> int {
    const int dx = x[b] - x[a], dy = y[b] - y[a], dz = z[b] - z[a];
    if (dx == 1 && dy == 0 && dz == 0) return 0;
    if (dx == 0 && dy == 1 && dz == 0) return 1;
    if (dx == 0 && dy == 0 && dz == 1) return 2;
    return -1;
  };
  const int a0 = axis(0, 1), a1 = axis(1, 2), a2 = axis(2, 3);
  int type = 7;
  if (a0 >= 0 && a1 >= 0 && a2 >= 0 && a0 != a1 && a1 != a2 && a0 != a2) {
    const int tbl[3][3] = { { -1, 0, 1 }, { 2, -1, 3 }, { 4, 5, -1 } };  // (a0, a1) -> c_kuhn index
    type = tbl[a0][a1];
  }
  keys[c] = (unsigned long long)(mx + L0 * (my + L1 * (int64_t)mz)) << 3 | (unsigned long long)type;
  ids[c] = (int32_t)c;
}

// the relabeled cells, each one's vertices in increasing lattice index (the
// generator's Kuhn path order, whatever the caller's vertex order)
__global__ void k_relabel_cells(int64_t nc, const int32_t* __restrict__ cn, const int32_t* __restrict__ order,
                                const int32_t* __restrict__ lat, int32_t* __restrict__ out)
{
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nc) return;
  int32_t v[4];
  for (int a = 0; a < 4; ++a) v[a] = lat[cn[4 * (int64_t)order[c] + a]];
  for (int i = 1; i < 4; ++i)
    for (int j = i; j > 0 && v[j] < v[j - 1]; --j) {
      const int32_t t = v[j];
      v[j] = v[j - 1];
      v[j - 1] = t;
    }
  for (int a = 0; a < 4; ++a) out[4 * c + a] = v[a];
}

__global__ void k_permute_coords(int64_t n, const int32_t* __restrict__ inv, const double* __restrict__ in,
                                 double* __restrict__ out)
{
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 3 * n) return;
  out[t] = in[3 * (int64_t)inv[t / 3] + t % 3];
}

__global__ void k_map_ids(int64_t n, const int32_t* __restrict__ inv, int32_t* __restrict__ v)
{
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n && v[t] >= 0) v[t] = inv[v[t]];
}

// physical row offsets and slot maps of the processing positions: canonical
// row R (lattice index) = node r; canonical slot t of R (its columns sorted by
// lattice index) -> the position of that column in r's id-sorted columns
__global__ void k_canon_slots(int64_t n_pos, const int32_t* __restrict__ perm_lat, const int32_t* __restrict__ inv,
                              const int64_t* __restrict__ crp, const int32_t* __restrict__ ccols,
                              const int64_t* __restrict__ rp, const int32_t* __restrict__ cols,
                              int64_t* __restrict__ pos_rb, uint8_t* __restrict__ cperm, int32_t* __restrict__ err)
{
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pos) return;
  uint8_t out[16] = {};
  const int32_t R = perm_lat[p];
  int64_t rb = 0;
  if (R >= 0) {
    const int32_t r = inv[R];
    rb = rp[r];
    const int len = (int)(rp[r + 1] - rb);
    const int64_t cb = crp[R];
    if (len != (int)(crp[R + 1] - cb) || len > 16) {
      *err = 1;
    }
    else {
      for (int t = 0; t < len; ++t) {
        const int q = find_slot(cols + rb, len, inv[ccols[cb + t]]);
        if (q >= len || cols[rb + q] != inv[ccols[cb + t]]) *err = 1;
        out[t] = (uint8_t)q;
      }
    }
  }
  pos_rb[p] = rb;
  for (int t = 0; t < 16; ++t) cperm[16 * p + t] = out[t];
}

// every cell a Kuhn tet (type < 6) and no two alike in one cube (sorted keys)
__global__ void k_kuhn_check(int64_t nc, const unsigned long long* __restrict__ keys, int32_t* __restrict__ err)
{
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nc) return;
  if ((keys[c] & 7ull) >= 6ull || (c > 0 && keys[c] == keys[c - 1])) *err = 1;
}

// the cube kernel's maps per lattice node i (canonical row i = the caller's
// row inv[i]): that row's first value and, per canonical slot t (columns
// sorted by lattice index), the position of the column in the caller's row
__global__ void k_cube_maps(int64_t n, const int32_t* __restrict__ inv, const int64_t* __restrict__ crp,
                            const int32_t* __restrict__ ccols, const int64_t* __restrict__ rp,
                            const int32_t* __restrict__ cols, int64_t* __restrict__ rb_out,
                            uint64_t* __restrict__ slot_out, int32_t* __restrict__ err)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t r = inv[i];
  const int64_t rb = rp[r];
  const int len = (int)(rp[r + 1] - rb);
  const int64_t cb = crp[i];
  uint64_t w = 0;
  if (len != (int)(crp[i + 1] - cb) || len > 15) {
    *err = 1;
  }
  else {
    for (int t = 0; t < len; ++t) {
      const int32_t c = inv[ccols[cb + t]];
      const int q = find_slot(cols + rb, len, c);
      if (q >= len || cols[rb + q] != c) *err = 1;
      w |= (uint64_t)(q & 15) << (4 * t);
    }
  }
  rb_out[i] = rb;
  slot_out[i] = w;
}

// axis orders of a lexicographic numbering, fastest axis first
constexpr int kAxisOrders[6][3] = { { 0, 1, 2 }, { 0, 2, 1 }, { 1, 0, 2 }, { 1, 2, 0 }, { 2, 0, 1 }, { 2, 1, 0 } };

// ---- natural lattice numberings.  A cartesian mesh handed over as arrays
// (Arcane's cartesian generator, a caller's own lexicographic loops) numbers
// its nodes lexicographically: id = l_a + L_a (l_b + L_b l_c) for some order
// (a, b, c) of the axes.  Up to that axis order this is the generator's box:
// the cube kernel runs on the caller's arrays with no map, when every cell is
// one of the 6 Kuhn tets of its lattice cube (the 6 tets of a cube are the 6
// axis permutations of the path from its lower to its upper corner, a set
// that does not depend on the axis order).

// bit q of *bad: node i is not at lexicographic index i in axis order q
__global__ void k_natural_ids(int64_t n, const int32_t* __restrict__ lx, const int32_t* __restrict__ ly,
                              const int32_t* __restrict__ lz, int64_t L0, int64_t L1, int64_t L2,
                              int32_t* __restrict__ bad)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t l[3] = { lx[i], ly[i], lz[i] };
  const int64_t L[3] = { L0, L1, L2 };
  int32_t b = 0;
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    const int a = kAxisOrders[q][0], c = kAxisOrders[q][1], d = kAxisOrders[q][2];
    if (l[a] + L[a] * (l[c] + L[c] * l[d]) != i) b |= 1 << q;
  }
  if (b) atomicOr(bad, b);
}

// every cell a Kuhn tet of its lattice cube, no cube holding one twice
// (with 6 cells per cube: each cube holds all six)
__global__ void k_kuhn_cubes(int64_t nc, const int32_t* __restrict__ cn, const int32_t* __restrict__ lx,
                             const int32_t* __restrict__ ly, const int32_t* __restrict__ lz, int64_t L0, int64_t L1,
                             int32_t* __restrict__ seen, int32_t* __restrict__ err)
{
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nc) return;
  int x[4], y[4], z[4];
  int mx = 1 << 30, my = 1 << 30, mz = 1 << 30;
  for (int a = 0; a < 4; ++a) {
    const int32_t v = cn[4 * c + a];
    x[a] = lx[v];
    y[a] = ly[v];
    z[a] = lz[v];
    mx = min(mx, x[a]);
    my = min(my, y[a]);
    mz = min(mz, z[a]);
  }
  // a Kuhn path climbs every lexicographic index at each step: sort by one
  auto lid = [&](int a) { return (int64_t)x[a] + L0 * ((int64_t)y[a] + L1 * (int64_t)z[a]); };
  for (int i = 1; i < 4; ++i)
    for (int j = i; j > 0 && lid(j) < lid(j - 1); --j) {
      const int tx = x[j], ty = y[j], tz = z[j];
      x[j] = x[j - 1];
      y[j] = y[j - 1];
      z[j] = z[j - 1];
      x[j - 1] = tx;
      y[j - 1] = ty;
      z[j - 1] = tz;
    }
  auto axis = [&](int a, int b) -> int {
    const int dx = x[b] - x[a], dy = y[b] - y[a], dz = z[b] - z[a];
    if (dx == 1 && dy == 0 && dz == 0) return 0;
    if (dx == 0 && dy == 1 && dz == 0) return 1;
    if (dx == 0 && dy == 0 && dz == 1) return 2;
    return -1;
  };
  const int a0 = axis(0, 1), a1 = axis(1, 2), a2 = axis(2, 3);
  if (a0 < 0 || a1 < 0 || a2 < 0 || a0 == a1 || a1 == a2 || a0 == a2 || mx + 1 >= L0 || my + 1 >= L1) {
    *err = 1;
    return;
  }
  const int bit = 1 << (3 * a0 + a1);
  const int64_t cube = mx + (L0 - 1) * (my + (L1 - 1) * (int64_t)mz);
  if (atomicOr(&seen[cube], bit) & bit) *err = 1;
}

// s.cube_natural (and the axis order) when the mesh is such a lattice
bool natural_lattice(Mesh& m, Structure& s)
{
  Ctx& ctx = *m.ctx;
  const int64_t n = s.n_rows;
  DevBuf<int32_t> lat3[3];
  int64_t L[3];
  if (!lattice_coords(ctx, m, n, lat3, L)) return false;
  const int64_t nc = m.n_cells;
  const int64_t n_cubes = (L[0] - 1) * (L[1] - 1) * (L[2] - 1);
  if (nc != 6 * n_cubes || nc == 0 || n > (int64_t)INT32_MAX) return false;
  DevBuf<int32_t> flags, seen;
  flags.alloc(2);
  seen.alloc(n_cubes);
  AFEM_HIP(hipMemsetAsync(flags.p, 0, flags.bytes(), ctx.stream));
  AFEM_HIP(hipMemsetAsync(seen.p, 0, seen.bytes(), ctx.stream));
  hipLaunchKernelGGL(k_natural_ids, dim3(grid_for(n, 256)), dim3(256), 0, ctx.stream, n, lat3[0].p, lat3[1].p,
                     lat3[2].p, L[0], L[1], L[2], flags.p);
  AFEM_LAUNCHED();
  hipLaunchKernelGGL(k_kuhn_cubes, dim3(grid_for(nc, 256)), dim3(256), 0, ctx.stream, nc, m.cell_node.p, lat3[0].p,
                     lat3[1].p, lat3[2].p, L[0], L[1], seen.p, flags.p + 1);
  AFEM_LAUNCHED();
  int32_t h[2] = { 0, 0 };
  AFEM_HIP(hipMemcpyAsync(h, flags.p, sizeof(h), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  if (h[1] != 0) return false;
  for (int q = 0; q < 6; ++q)
    if (!((h[0] >> q) & 1)) {
      s.cube_natural = true;
      for (int a = 0; a < 3; ++a) {
        s.nat_axes[a] = kAxisOrders[q][a];
        s.nat_L[a] = L[kAxisOrders[q][a]];
      }
      return true;
    }
  return false;
}

// the canonical structure of a lattice mesh (see above) into s; false when it
// does not apply or does not reach the stencil instance
bool canonical_lattice(Mesh& m, Structure& s)
{
  Ctx& ctx = *m.ctx;
  const int64_t n = s.n_rows;
  DevBuf<int32_t> lat3[3];
  int64_t L[3];
  if (!lattice_coords(ctx, m, n, lat3, L)) return false;
  DevBuf<int32_t> lat, inv;
  lat.alloc(n);
  inv.alloc(n);
  hipLaunchKernelGGL(k_lat_ids, dim3(grid_for(n, 256)), dim3(256), 0, ctx.stream, n, lat3[0].p, lat3[1].p, lat3[2].p,
                     L[0], L[1], lat.p, inv.p);
  AFEM_LAUNCHED();
  // the relabeled mesh: lattice node ids, cells in the generator's order
  const int64_t nc = m.n_cells;
  bool kuhn = false;
  Mesh R;
  R.ctx = m.ctx;
  R.dim = 3;
  R.nv = 4;
  R.n_nodes = R.n_own = n;
  R.n_cells = nc;
  R.cell_node.alloc(4 * nc);
  R.coords.alloc(3 * n);
  {
    DevBuf<unsigned long long> keys, keys_s;
    DevBuf<int32_t> ids, ids_s;
    keys.alloc(nc);
    keys_s.alloc(nc);
    ids.alloc(nc);
    ids_s.alloc(nc);
    hipLaunchKernelGGL(k_cell_keys, dim3(grid_for(nc, 256)), dim3(256), 0, ctx.stream, nc, m.cell_node.p, lat3[0].p,
                       lat3[1].p, lat3[2].p, L[0], L[1], keys.p, ids.p);
    AFEM_LAUNCHED();
    size_t tmp_bytes = 0;
    AFEM_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, keys.p, keys_s.p, ids.p, ids_s.p, (int)nc, 0, 64,
                                                ctx.stream));
    DevBuf<unsigned char> tmp;
    tmp.alloc(tmp_bytes > 0 ? tmp_bytes : 1);
    AFEM_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.p, tmp_bytes, keys.p, keys_s.p, ids.p, ids_s.p, (int)nc, 0, 64,
                                                ctx.stream));
    hipLaunchKernelGGL(k_relabel_cells, dim3(grid_for(nc, 256)), dim3(256), 0, ctx.stream, nc, m.cell_node.p,
                       ids_s.p, lat.p, R.cell_node.p);
    AFEM_LAUNCHED();
    // the cube kernel needs the generator's cells: 6 distinct Kuhn tets per lattice cube
    const int64_t n_cubes = (L[0] - 1) * (L[1] - 1) * (L[2] - 1);
    kuhn = nc == 6 * n_cubes && nc > 0;
    if (kuhn) {
      DevBuf<int32_t> kerr;
      kerr.alloc(1);
      AFEM_HIP(hipMemsetAsync(kerr.p, 0, kerr.bytes(), ctx.stream));
      hipLaunchKernelGGL(k_kuhn_check, dim3(grid_for(nc, 256)), dim3(256), 0, ctx.stream, nc, keys_s.p, kerr.p);
      AFEM_LAUNCHED();
      int32_t h = 0;
      AFEM_HIP(hipMemcpyAsync(&h, kerr.p, sizeof(h), hipMemcpyDeviceToHost, ctx.stream));
      ctx.sync();
      kuhn = h == 0;
    }
  }
  hipLaunchKernelGGL(k_permute_coords, dim3(grid_for(3 * n, 256)), dim3(256), 0, ctx.stream, n, inv.p, m.coords.p,
                     R.coords.p);
  AFEM_LAUNCHED();
  R.st.valid = true;
  R.st.dim = 3;
  R.st.n = (int)(L[0] - 1);
  R.st.lx = L[0];
  R.st.ly = L[1];
  R.st.nz = (int)(L[2] - 1);
  R.st.k0 = 0;
  R.st.k1 = (int)L[2];
  R.st.L = L[0] * L[1];
  Structure C;
  build_structure_impl(R, C);
  if (!C.strip_ok || !C.rec_ok || C.n_k == 0 || C.n_mb > 0 || C.max_strip_c > 2 || C.max_slice_w > 16 ||
      C.nnz != s.nnz)
    return false;
  // back to the caller's numbering: node ids of the positions and node lists,
  // physical row offsets, slot maps
  const int64_t n_pos = C.n_slices * 64;
  DevBuf<int32_t> perm_lat;
  perm_lat.alloc(n_pos);
  AFEM_HIP(hipMemcpyAsync(perm_lat.p, C.perm.p, perm_lat.bytes(), hipMemcpyDeviceToDevice, ctx.stream));
  C.cperm.alloc(16 * n_pos);
  DevBuf<int32_t> err;
  err.alloc(1);
  AFEM_HIP(hipMemsetAsync(err.p, 0, err.bytes(), ctx.stream));
  hipLaunchKernelGGL(k_canon_slots, dim3(grid_for(n_pos, 256)), dim3(256), 0, ctx.stream, n_pos, perm_lat.p, inv.p,
                     C.row_ptr.p, C.cols.p, s.row_ptr.p, s.cols.p, C.pos_rb.p, C.cperm.p, err.p);
  AFEM_LAUNCHED();
  hipLaunchKernelGGL(k_map_ids, dim3(grid_for(n_pos, 256)), dim3(256), 0, ctx.stream, n_pos, inv.p, C.perm.p);
  AFEM_LAUNCHED();
  hipLaunchKernelGGL(k_map_ids, dim3(grid_for((int64_t)C.snode.n, 256)), dim3(256), 0, ctx.stream,
                     (int64_t)C.snode.n, inv.p, C.snode.p);
  AFEM_LAUNCHED();
  // the cube kernel's maps (while C's row structure is still the canonical one)
  if (kuhn) {
    C.cube_phys.alloc(n);
    C.cube_rb.alloc(n);
    C.cube_slot.alloc(n);
    AFEM_HIP(hipMemcpyAsync(C.cube_phys.p, inv.p, C.cube_phys.bytes(), hipMemcpyDeviceToDevice, ctx.stream));
    DevBuf<int32_t> cerr;
    cerr.alloc(1);
    AFEM_HIP(hipMemsetAsync(cerr.p, 0, cerr.bytes(), ctx.stream));
    hipLaunchKernelGGL(k_cube_maps, dim3(grid_for(n, 256)), dim3(256), 0, ctx.stream, n, inv.p, C.row_ptr.p, C.cols.p,
                       s.row_ptr.p, s.cols.p, C.cube_rb.p, C.cube_slot.p, cerr.p);
    AFEM_LAUNCHED();
    int32_t h = 0;
    AFEM_HIP(hipMemcpyAsync(&h, cerr.p, sizeof(h), hipMemcpyDeviceToHost, ctx.stream));
    ctx.sync();
    C.cube_ok = h == 0;
    for (int a = 0; a < 3; ++a) C.cube_L[a] = L[a];
  }
  int32_t herr = 0;
  AFEM_HIP(hipMemcpyAsync(&herr, err.p, sizeof(herr), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  if (herr) return false;
  // the matrix structure stays the caller's; everything else is the canonical build
  C.row_ptr = std::move(s.row_ptr);
  C.cols = std::move(s.cols);
  C.diag_pos = std::move(s.diag_pos);
  C.n_rows = s.n_rows;
  C.n_cols = s.n_cols;
  C.nnz = s.nnz;
  C.max_row_len = s.max_row_len;
  C.inc.reset();  // canonical slots: the incidence-table kernels are not used on this structure
  C.lattice = true;
  C.canon = true;
  s = std::move(C);
  return true;
}

}  // namespace

void build_structure(Mesh& m, Structure& s, int nb_dof)
{
  build_structure_impl(m, s);
  if (!(nb_dof == 1 && s.lattice && m.nv == 4 && m.dim == 3 && m.n_nodes == m.n_own)) return;
  // an array-fed Kuhn lattice in a natural numbering: the cube kernel as on
  // the generator's box (AFEM_CUBE_NATURAL=0: not)
  const char* ne = variant("AFEM_CUBE_NATURAL");
  if (!(ne && atoi(ne) == 0)) (void)natural_lattice(m, s);
  // an array-fed lattice whose numbering keeps it off the stencil instance
  // (for the strip kernels: a natural numbering in another axis order too)
  const char* ce = variant("AFEM_CANON");
  if (s.n_k * 2 < s.n_slices && s.max_row_len <= 16 && !(ce && atoi(ce) == 0)) {
    const bool nat = s.cube_natural;
    int ax[3];
    int64_t nl[3];
    for (int a = 0; a < 3; ++a) {
      ax[a] = s.nat_axes[a];
      nl[a] = s.nat_L[a];
    }
    if (canonical_lattice(m, s)) {
      s.cube_natural = nat;
      for (int a = 0; a < 3; ++a) {
        s.nat_axes[a] = ax[a];
        s.nat_L[a] = nl[a];
      }
    }
  }
}

}  // namespace afem
