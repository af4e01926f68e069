// Scalar P1 (Poisson) assembly on the generator's Kuhn boxes, cell first:
// k_assemble_cubes.
//
// The strip / stencil kernels (assembly.hip) are row first: each of a tet's 4
// rows walks its cells and recomputes the tet's geometry (two cross products,
// |det|, the reciprocal: ~50 FP64 operations per row-step, 24 steps per row).
// Here each cube of the lattice is evaluated ONCE per unit: its 6 Kuhn tets
// (mesh.hip c_kuhn: for each axis permutation (a0,a1,a2) the tet
// (v0, v0+e_a0, v0+e_a0+e_a1, v0+(1,1,1))) give the cofactors, |det| and the 6
// off-diagonal entries K_ab = coef c_a.c_b / (6|det|) once; the contributions
// of the 6 tets to each of the cube's 19 Kuhn edges are summed in registers
// and added to the two rows of the edge with ds_add_f64 (LDS, wave-local, in
// program order: deterministic), the |det| sums of each corner likewise (the
// RHS source f |det| / 24, fused).  ~600 VALU operations per cube against
// ~1500 per row for the strip kernels.
//
// Unit = one wavefront: a column of 7 x 7 rows (node lines) over zs owned node
// layers.  Lane (i, j) owns the cube with lower corner (cx0 - 1 + i,
// cy0 - 1 + j): the 8 x 8 cubes touching the column's 7 x 7 rows, one per lane
// (the halo cubes are evaluated by both neighbouring columns: 64/49 = 1.31
// evaluations per cube, plus 1/zs for the cube layer below a segment).  The
// unit walks the cube layers upwards: node layer z's rows take the cube layers
// z-1 and z, so two row-layer accumulator buffers (by parity) live in LDS,
// [15][STRIDE] doubles each (15 column offsets in sorted order; the diagonal's
// plane, never added to, holds the |det| sum),
// and the node coordinates of the two layers of the current cube layer
// (9 x 9 nodes each, staged from registers loaded one layer ahead).  When a
// node layer is complete its 49 rows are written once: the values compacted
// by each row's present neighbours into a flat LDS image, then each x-run of
// 7 rows (contiguous in the matrix) with consecutive lanes.
//
// Applies to meshes from afem_mesh_create_structured (3D, NB_DOF 1, any
// z-slab: the columns follow the local numbering -- owned layers, then the
// ghost layer below, then above -- so the sorted column order of a row next to
// the ghost layer below is recovered from the layers' local indices), and to
// lattices of Kuhn cubes handed over as arrays in any numbering (CANON: the
// structure's canonical maps, sparsity.hip canonical_lattice).  Values
// equal the oracle's to rounding (1e-12 per entry); not bitwise the strip
// kernels' (another summation order).  The default on generator boxes (C2:
// 0.58-0.59 ms against the stencil kernel's 0.64);
// AFEM_ASSEMBLY_CUBES=0 takes the strip / stencil path.
#include "afem_internal.hpp"

#include <algorithm>

// the 64-row instances cannot reach the 3-waves register target (their LDS
// allows 2 per SIMD): the compiler says so for each; expected
#pragma clang diagnostic ignored "-Wpass-failed"

namespace afem {

namespace {

inline unsigned grid_for(int64_t n, int threads) { return (unsigned)((n + threads - 1) / threads); }

struct P3 {
  double x, y, z;
};
__device__ __forceinline__ P3 psub(P3 a, P3 b) { return P3{ a.x - b.x, a.y - b.y, a.z - b.z }; }
__device__ __forceinline__ P3 pcross(P3 a, P3 b)
{
  return P3{ fma(a.y, b.z, -(a.z * b.y)), fma(a.z, b.x, -(a.x * b.z)), fma(a.x, b.y, -(a.y * b.x)) };
}
__device__ __forceinline__ double pdot(P3 a, P3 b) { return fma(a.z, b.z, fma(a.y, b.y, a.x * b.x)); }
__device__ __forceinline__ double precip(double a)
{
  const double r = __builtin_amdgcn_rcp(a);
  const double e = fma(-a, r, 1.0);
  return fma(r, e, r);
}

struct CubeGeom {
  int npx, npy;      // nodes per x line, per y line
  int nzc;           // cells of the global box in z (node layers 0..nzc)
  int k0, k1;        // owned node layers [k0, k1)
  int ghost_lo, ghost_hi;
  int n_own_layers;
  int64_t L;         // nodes per layer
  int tx, ty, zs, ns;
  double s_coef;     // coef / 6
  double f_meas;     // f / 24
  int full_flush;    // flush_full for layers whose rows are all complete (AFEM_CUBES_FULL=0: not)
};

// is global node layer k one of the slab's local layers (owned or ghost)?
__device__ __forceinline__ bool is_local(const CubeGeom& g, int k)
{
  return (k >= g.k0 && k < g.k1) || (k >= 0 && (k == g.ghost_lo || k == g.ghost_hi));
}
// local layer index of global node layer k (mesh.hip Layers::local_layer)
__device__ __forceinline__ int local_layer(const CubeGeom& g, int k)
{
  if (k >= g.k0 && k < g.k1) return k - g.k0;
  if (k == g.ghost_lo) return g.n_own_layers;
  return g.n_own_layers + (g.ghost_lo >= 0 ? 1 : 0);
}

// the 15 column offsets of a Kuhn row sorted by node id (x + npx (y + npy z)):
// by dz, then dy, then dx
__host__ __device__ constexpr int o_of(int dx, int dy, int dz)
{
  return dz < 0 ? (dy < 0 ? (dx < 0 ? 0 : 1) : (dx < 0 ? 2 : 3))
                : dz == 0 ? (dy < 0 ? (dx < 0 ? 4 : 5) : dy == 0 ? (dx < 0 ? 6 : (dx == 0 ? 7 : 8)) : (dx == 0 ? 9 : 10))
                          : (dy == 0 ? (dx == 0 ? 11 : 12) : (dx == 0 ? 13 : 14));
}
constexpr int kOffX[15] = { -1, 0, -1, 0, -1, 0, -1, 0, 1, 0, 1, 0, 1, 0, 1 };
constexpr int kOffY[15] = { -1, -1, 0, 0, -1, -1, 0, 0, 0, 1, 1, 0, 0, 1, 1 };
constexpr int kOffZ[15] = { -1, -1, -1, -1, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1 };

// corners c = ci + 2 cj + 4 ck; tet t = (0, 1 << a0, (1 << a0) | (1 << a1), 7)
constexpr int kPerm[6][2] = { { 0, 1 }, { 0, 2 }, { 1, 0 }, { 1, 2 }, { 2, 0 }, { 2, 1 } };
__host__ __device__ constexpr int tet_v(int t, int k)
{
  return k == 0 ? 0 : k == 1 ? (1 << kPerm[t][0]) : k == 2 ? ((1 << kPerm[t][0]) | (1 << kPerm[t][1])) : 7;
}
__host__ __device__ constexpr int cbit(int c, int a) { return (c >> a) & 1; }
// the row offset index of corner b seen from corner a
__host__ __device__ constexpr int edge_o(int a, int b)
{
  return o_of(cbit(b, 0) - cbit(a, 0), cbit(b, 1) - cbit(a, 1), cbit(b, 2) - cbit(a, 2));
}
// is (a, b), a < b, an edge of one of the 6 tets?
__host__ __device__ constexpr bool is_edge(int a, int b)
{
  bool e = false;
  for (int t = 0; t < 6; ++t)
    for (int p = 0; p < 4; ++p)
      for (int q = 0; q < 4; ++q)
        if (tet_v(t, p) == a && tet_v(t, q) == b) e = true;
  return e;
}

// lane L's value, wave-uniform (v_readlane into a scalar register: no LDS
// permute, and the address arithmetic on it stays scalar)
__device__ __forceinline__ int lane_i32(int v, int L) { return __builtin_amdgcn_readlane(v, L); }
__device__ __forceinline__ int64_t lane_i64(int64_t v, int L)
{
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, L);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), L);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double lane_f64(double v, int L) { return __longlong_as_double(lane_i64(__double_as_longlong(v), L)); }

constexpr int kRun = 7;    // rows per x-run of a column
constexpr int kRows = 49;  // rows per column layer
constexpr int kCol = 9;    // staged nodes per x / y line (the column's rows + 1 halo line below)
constexpr int kAcc = 15;   // accumulators per row: 15 offsets, the diagonal's (7, never added to:
                           // v_7 = -sum of the others) holds the row's |det| sum

// One wave per block: LDS operations of a wave execute in issue order, so
// ordering its phases (staging -> cube adds -> flush reads -> image -> stores)
// needs only the compiler to keep the order, not an lgkmcnt(0) drain as
// __syncthreads emits (AFEM_CUBES_WAVESYNC=0 restores those)
#ifndef AFEM_CUBES_WAVESYNC
#define AFEM_CUBES_WAVESYNC 1
#endif
__device__ __forceinline__ void wave_lds_order()
{
#if AFEM_CUBES_WAVESYNC
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
#else
  __syncthreads();
#endif
}

// a value store, non-temporal when NT (cubes: V bits 32 / 128)
template <bool NT>
__device__ __forceinline__ void put(double* p, double v)
{
  if constexpr (NT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// HAS_RHS / RHS_ADD at compile time: the flush's global stores are then a
// fixed, branch-free sequence, so the waits for the next layer's coordinates
// count past them (vmcnt(N)) instead of draining them (vmcnt(0))
// amdgpu_waves_per_eu(3): 168 VGPRs, with the 49-row planes' 15.6 KB of LDS
// 10 waves per CU (the 64-row planes' 19.3 KB keep 8 whatever the registers)
// CANON: a lattice mesh in the caller's numbering (sparsity.hip canonical_lattice,
// Structure::cube_*): the unit walks lattice indices; a node's coordinates
// come through its caller id, a row's values go to the caller's row (first
// value cc.rb, canonical slot t at position cc.slot >> 4t) through a per-row
// image (row L at [15 L, 15 L + 15), stored row by row)
struct CubeCanon {
  const int32_t* phys;
  const int64_t* rb;
  const uint64_t* slot;
  double* stage;  // STAGE: one 128-B line per lattice row
};

// V: variant bits (AFEM_CUBES_V; the default kCubesV is what every result
// uses).  Values right: 16 the next layer's coordinates loaded before the
// cubes (their latency hides behind them), 32 non-temporal value stores in
// the complete-layer flush (the values are not re-read by this launch; the
// L2 keeps the coordinates the neighbouring units re-read), 64 one 16-B
// store per lane and x-run there (7 stores per layer instead of 14), 128
// non-temporal value and RHS stores in the other flushes, 256 dummy rows for
// the corners outside the unit (no zero selects; 64-row planes), 512 16-B
// row stores in the canonical flush, 1024 the canonical path STAGED (its rows
// written in lattice order as one 128-B line each -- the 15 values by Kuhn
// offset, the |det| sum at 15 -- and moved into the caller's rows by
// k_cube_unstage, caller row by caller row: whole-line stores).  Diagnostic
// ablations (values wrong): 1 no value stores in the complete-layer flush, 2
// one LDS add per cube (the sum of its sums) instead of its 15, 4 no cube
// arithmetic, 8 no complete-layer flush.  Measured (r05d/e, C2 / C4, one
// process, settled): 0.520 / 4.53 ms with none, 0.465 / 4.20 with 16 | 32 | 64;
// adding 128 costs 5.6 % on the box and 11 % on the random arrays (r05h:
// scattered 8-B RHS stores and 120-B rows are worse non-temporal); 256 on top
// of 16 | 32 | 64: C2 0.4632 -> 0.4608 ms, C4 4.194 -> 4.097 ms (r05i); 512:
// random-numbered arrays (canonical path) 1.581 -> 1.538 ms (r05k); 1024 there:
// 1.539 -> 1.103 ms (r05as: 0.587 ms cube pass + 0.532 ms k_cube_unstage).
constexpr int kCubesV = 16 | 32 | 64 | 256 | 512 | 1024;

// register budget: 64-row planes + one coordinate layer = 17.3 KB of LDS, 9
// waves per CU, so 2 per SIMD whatever the registers (256 VGPRs, no spill);
// 49-row planes = 13.7 KB, 11 waves per CU: 3 per SIMD at <= 168 VGPRs
template <int STRIDE>
constexpr int cube_waves() { return STRIDE == 64 ? 2 : 3; }
template <int STRIDE, bool CARRY, bool XEX, bool YEX, bool CANON, bool HAS_RHS, bool RHS_ADD, int DIAG = kCubesV>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(cube_waves<STRIDE>(), cube_waves<STRIDE>()))) void k_assemble_cubes(
    CubeGeom g, const int64_t* __restrict__ rows, const double* __restrict__ coords, double* __restrict__ vals,
    double* __restrict__ rhs, CubeCanon cc)
{
  __shared__ __align__(16) double acc[2][kAcc][STRIDE];  // STRIDE >= 49 rows per offset plane
  // SoA coordinates of the node layers being read: with the carry the bottom
  // corners come from registers (Xc), so one layer -- the cube layer's top --
  // is read, and the next one is staged over it after the cubes
  constexpr int NCZ = CARRY ? 1 : 2;
  __shared__ double cz[NCZ][3][kCol * kCol];
  const int lane = threadIdx.x;
  // XCD-aware: blocks go round-robin over the 8 XCDs; XCD x takes the x-th
  // contiguous eighth of the units (x fastest, then y, then segments)
  const int64_t n_units = (int64_t)g.tx * g.ty * g.ns;
  const int64_t bid = blockIdx.x;
  const int64_t qq = n_units >> 3, rem = n_units & 7, xc = bid & 7, jj = bid >> 3;
  const int64_t u = xc * qq + (xc < rem ? xc : rem) + jj;
  const int utx = (int)(u % g.tx);
  const int uty = (int)((u / g.tx) % g.ty);
  const int seg = (int)(u / ((int64_t)g.tx * g.ty));
  const int cx0 = kRun * utx, cy0 = kRun * uty;
  const int z0 = g.k0 + seg * g.zs;
  const int z1 = min(z0 + g.zs, g.k1);
  const int zc_first = max(z0 - 1, 0);
  const int zc_last = min(z1 - 1, g.nzc - 1);  // cube layer zc: node layers zc, zc + 1

  // this lane's cube (i, j) and its staging share (nodes q = lane, lane + 64 of 81)
  const int ci = lane & 7, cj = lane >> 3;
  const int gx = cx0 - 1 + ci, gy = cy0 - 1 + cj;  // lower corner
  const bool cube_in = gx >= 0 && gy >= 0 && gx + 1 < g.npx && gy + 1 < g.npy;
  auto node_xy = [&](int q, int& nx, int& ny) {
    nx = cx0 - 1 + q % kCol;
    ny = cy0 - 1 + q / kCol;
  };
  // staging loads without branches (addresses clamped into the local mesh,
  // out-of-range positions hold a duplicate that no cube reads): straight-line
  // code, so the waits on them count past the later memory operations instead
  // of draining everything (vmcnt(0)) at a branch join
  double pre[2][3];
  int32_t pid[2] = { 0, 0 };  // CANON: the caller's ids of the next staged layer's nodes
  auto layer_ids = [&](int k, int64_t(&id)[2]) {
    const int kk = is_local(g, k) ? k : g.k0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int q = min(lane + 64 * h, kCol * kCol - 1);
      int nx, ny;
      node_xy(q, nx, ny);
      nx = min(max(nx, 0), g.npx - 1);
      ny = min(max(ny, 0), g.npy - 1);
      id[h] = (int64_t)local_layer(g, kk) * g.L + nx + (int64_t)g.npx * ny;
    }
  };
  // CANON: the ids first (prefetch_ids, one step ahead), the coordinates through them
  auto prefetch_ids = [&](int k) {
    if constexpr (CANON) {
      int64_t id[2];
      layer_ids(k, id);
#pragma unroll
      for (int h = 0; h < 2; ++h) pid[h] = cc.phys[id[h]];
    }
  };
  auto load_layer = [&](int k) {
    int64_t id[2];
    layer_ids(k, id);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t n = CANON ? (int64_t)pid[h] : id[h];
      pre[h][0] = coords[3 * n];
      pre[h][1] = coords[3 * n + 1];
      pre[h][2] = coords[3 * n + 2];
    }
  };
  auto store_layer = [&](int buf) {
    buf = NCZ == 1 ? 0 : buf;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int q = min(lane + 64 * h, kCol * kCol - 1);  // lanes past the 81 nodes repeat node 80's store
      cz[buf][0][q] = pre[h][0];
      cz[buf][1][q] = pre[h][1];
      cz[buf][2][q] = pre[h][2];
    }
  };
  for (int i = lane; i < 2 * kAcc * STRIDE; i += 64) (&acc[0][0][0])[i] = 0.0;

  // ---- node layer z complete: write its 49 rows (values compacted by the present neighbours) + RHS.
  // The rows' offsets are loaded before the layer's cubes (prefetch_rows), so
  // their latency hides behind the cube arithmetic instead of stalling here.
  const int rx = lane % kRun, ry = lane / kRun;
  const int nx = cx0 + rx, ny = cy0 + ry;
  const bool full_flush_on = g.full_flush != 0;
  constexpr bool STAGE = CANON && (DIAG & 1024) != 0;
  int64_t pf_rb = 0, pf_re = 0, pf_r = 0;
  uint64_t pf_slot = 0;
  double pf_rhs = 0.0;
  auto prefetch_rows = [&](int z) {  // clamped like load_layer: no branch
    const int zz = (z >= z0 && z < z1) ? z : z0;
    const int64_t li = (int64_t)local_layer(g, zz) * g.L + min(nx, g.npx - 1) + (int64_t)g.npx * min(ny, g.npy - 1);
    if constexpr (STAGE) {
      (void)li;  // the rows' maps are k_cube_unstage's
    }
    else if constexpr (CANON) {
      pf_r = cc.phys[li];
      pf_rb = cc.rb[li];
      pf_slot = cc.slot[li];
    }
    else {
      pf_r = li;
      pf_rb = rows[pf_r];
      pf_re = rows[pf_r + 1];
      if constexpr (RHS_ADD) pf_rhs = rhs[pf_r];
    }
  };
  // a node layer whose 49 rows all have their 15 neighbours, in the sorted
  // order of the offsets (the unit away from the x / y faces of the box, z
  // off its bottom and top layers, the local layers in id order: not next to
  // a slab's ghost layer below): the row's values go to the image at 15 L + o,
  // and each x-run is 105 consecutive image values -- no masks, no
  // compaction, constant LDS offsets (flush_full)
  const bool xy_full = cx0 >= 1 && cx0 + kRun <= g.npx - 1 && cy0 >= 1 && cy0 + kRun <= g.npy - 1;
  auto layer_full = [&](int z) {
    return xy_full && z >= 1 && z + 1 <= g.nzc && local_layer(g, z - 1) < local_layer(g, z) &&
           local_layer(g, z) < local_layer(g, z + 1);
  };
  auto flush_full = [&](int z) {
    const int b = z & 1;
    const int lr = min(lane, STRIDE - 1);  // lanes past the 49 rows read a row they do not use
    double v[15];
    double sum = 0.0;
#pragma unroll
    for (int o = 0; o < 15; ++o) {
      v[o] = acc[b][o][lr];
      if (o != 7) sum += v[o];
    }
    const double meas = v[7];
    v[7] = -sum;
    if constexpr (HAS_RHS) {  // lanes without a row repeat lane 0's store
      const bool valid = lane < kRows;
      const double rv = RHS_ADD ? pf_rhs + g.f_meas * meas : g.f_meas * meas;
      const int64_t r0 = lane_i64(pf_r, 0);
      const double rv0 = lane_f64(rv, 0);
      put<(DIAG & 128) != 0>(&rhs[valid ? pf_r : r0], valid ? rv : rv0);
    }
    const int64_t rb = pf_rb;
    double* img = &acc[b][0][0];
    // (each lane storing its own row from registers instead -- 7 16-B stores at a
    // 120-B lane stride -- measured 3.19 against 0.456 ms, r05aw: the image stays)
    wave_lds_order();  // every lane's accumulator reads before the image overwrites them
    // row L at [15 L, 15 L + 15): lanes past the 49 rows write into
    // [735, 960) of the buffer, which no store reads (64-row planes), or --
    // 49-row planes, whose buffer ends at 735 -- repeat row 48's writes with
    // row 48's values (they read row 48: same addresses, same values)
#pragma unroll
    for (int o = 0; o < 15; ++o) img[15 * (STRIDE == 64 ? lane : lr) + o] = v[o];
    wave_lds_order();
    // x-run q = rows 7q .. 7q + 6: 105 values contiguous in vals from row 7q's
    // first one; the second store's lanes past 105 repeat value 104 (same
    // address, same value)
    const int t1 = min(lane + 64, 15 * kRun - 1);
    // DIAG 64: one 16-B store per lane and run (values 2l, 2l + 1; lane 52
    // stores 103, 104 -- value 103 twice with the same data -- and the lanes
    // past it repeat lane 52's): 7 stores per layer instead of 14
    const int t2 = min(2 * lane, 15 * kRun - 2);
#pragma unroll
    for (int q = 0; q < kRun; ++q) {
      const int64_t dst = lane_i64(rb, kRun * q);
      if constexpr ((DIAG & 1) != 0) {
        (void)dst;  // diagnostic: no value stores
      }
      else if constexpr ((DIAG & 64) != 0) {
        const double a0 = img[15 * kRun * q + t2], a1 = img[15 * kRun * q + t2 + 1];
        typedef double d2u __attribute__((ext_vector_type(2), aligned(8)));
        if constexpr ((DIAG & 32) != 0)
          __builtin_nontemporal_store(d2u{ a0, a1 }, reinterpret_cast<d2u*>(&vals[dst + t2]));
        else
          *reinterpret_cast<d2u*>(&vals[dst + t2]) = d2u{ a0, a1 };
      }
      else if constexpr ((DIAG & 32) != 0) {
        __builtin_nontemporal_store(img[15 * kRun * q + lane], &vals[dst + lane]);
        __builtin_nontemporal_store(img[15 * kRun * q + t1], &vals[dst + t1]);
      }
      else {
        vals[dst + lane] = img[15 * kRun * q + lane];
        vals[dst + t1] = img[15 * kRun * q + t1];
      }
    }
    wave_lds_order();
    if constexpr ((kAcc * STRIDE) % 2 == 0) {
      double2* const img2 = reinterpret_cast<double2*>(img);
#pragma unroll
      for (int i = 0; i < (kAcc * STRIDE / 2 + 63) / 64; ++i)
        img2[min(64 * i + lane, kAcc * STRIDE / 2 - 1)] = make_double2(0.0, 0.0);
    }
    else {
#pragma unroll
      for (int i = 0; i < (kAcc * STRIDE + 63) / 64; ++i) img[min(64 * i + lane, kAcc * STRIDE - 1)] = 0.0;
    }
    wave_lds_order();
  };
  // STAGE: node layer z's rows into their lattice-order lines, line L = the
  // row's 15 values by Kuhn offset o and its |det| sum at 15 (an absent
  // neighbour's value is the zero its slot holds and is never moved); x-run q
  // = 7 lines = 112 consecutive doubles, one 16-B non-temporal store per lane
  auto flush_stage = [&](int z) {
    const int b = z & 1;
    const bool valid = lane < kRows && nx < g.npx && ny < g.npy;
    uint32_t mask = 0;
#pragma unroll
    for (int o = 0; o < 15; ++o) {
      const int xx = nx + kOffX[o], yy = ny + kOffY[o], zz = z + kOffZ[o];
      const uint32_t in = (uint32_t)(xx >= 0) & (uint32_t)(yy >= 0) & (uint32_t)(xx < g.npx) & (uint32_t)(yy < g.npy) &
                          (uint32_t)(zz >= 0) & (uint32_t)(zz <= g.nzc);
      mask |= in << o;
    }
    if (!valid) mask = 0;
    double v[15];
    double sum = 0.0;
    const int lr = min(lane, STRIDE - 1);
#pragma unroll
    for (int o = 0; o < 15; ++o) {
      v[o] = acc[b][o][lr];
      if (o != 7 && ((mask >> o) & 1u)) sum += v[o];
    }
    const double meas = v[7];
    v[7] = -sum;
    wave_lds_order();  // every lane's accumulator reads before the image overwrites them
    double* img = &acc[b][0][0];
    if (lane < kRows) {  // 49 lines of 16 = 784 of the buffer's 960 doubles
#pragma unroll
      for (int o = 0; o < 15; ++o) img[16 * lane + o] = v[o];
      img[16 * lane + 15] = meas;
    }
    wave_lds_order();
    typedef double d2u __attribute__((ext_vector_type(2), aligned(16)));
    const int64_t lz = (int64_t)local_layer(g, z) * g.L + cx0;
    const bool xok = lane < 2 * 8 * kRun / 2 && cx0 + (lane >> 3) < g.npx;  // pair `lane` is line lane / 8's
#pragma unroll
    for (int q = 0; q < kRun; ++q) {
      if (cy0 + q >= g.npy) break;  // uniform
      // lanes without a line repeat lane 0's pair (same address, same values)
      const int t = xok ? 2 * lane : 0;
      const d2u w = d2u{ img[2 * 8 * kRun * q + t], img[2 * 8 * kRun * q + t + 1] };
      __builtin_nontemporal_store(w, reinterpret_cast<d2u*>(&cc.stage[16 * (lz + (int64_t)g.npx * (cy0 + q)) + t]));
    }
    wave_lds_order();
    double2* const img2 = reinterpret_cast<double2*>(img);
#pragma unroll
    for (int i = 0; i < (kAcc * STRIDE / 2 + 63) / 64; ++i)
      img2[min(64 * i + lane, kAcc * STRIDE / 2 - 1)] = make_double2(0.0, 0.0);
    wave_lds_order();
  };
  auto flush = [&](int z) {
    if constexpr (STAGE) {
      flush_stage(z);
      return;
    }
    if constexpr (!CANON) {
      if (full_flush_on && layer_full(z)) {
        if constexpr (!(DIAG & 8)) flush_full(z);
        return;
      }
    }
    const int b = z & 1;
    const bool valid = lane < kRows && nx < g.npx && ny < g.npy;
    // present neighbours and the order of their local ids: the dz groups by local layer index
    uint32_t mask = 0;
#pragma unroll
    for (int o = 0; o < 15; ++o) {  // branch-free (bitwise ands of the comparisons)
      const int xx = nx + kOffX[o], yy = ny + kOffY[o], zz = z + kOffZ[o];
      const uint32_t in = (uint32_t)(xx >= 0) & (uint32_t)(yy >= 0) & (uint32_t)(xx < g.npx) & (uint32_t)(yy < g.npy) &
                          (uint32_t)(zz >= 0) & (uint32_t)(zz <= g.nzc);
      mask |= in << o;
    }
    if (!valid) mask = 0;
    const uint32_t gm0 = mask & 0x000Fu, gm1 = mask & 0x07F0u, gm2 = mask & 0x7800u;
    const int lm = local_layer(g, z - 1), l0 = local_layer(g, z), lp = local_layer(g, z + 1);
    const int n0 = __popc(gm0), n1 = __popc(gm1), n2 = __popc(gm2);
    const int s0 = (l0 < lm ? n1 : 0) + (lp < lm ? n2 : 0);
    const int s1 = (lm < l0 ? n0 : 0) + (lp < l0 ? n2 : 0);
    const int s2 = (lm < lp ? n0 : 0) + (l0 < lp ? n1 : 0);
    double v[15];
    double sum = 0.0;
    const int lr = min(lane, STRIDE - 1);  // lanes past the 49 rows read a row they do not use
#pragma unroll
    for (int o = 0; o < 15; ++o) {
      v[o] = acc[b][o][lr];
      if (o != 7 && ((mask >> o) & 1u)) sum += v[o];
    }
    const double meas = v[7];
    v[7] = -sum;
    // the prefetched offsets are consumed without a branch (selects), so the
    // compiler keeps their load where prefetch_rows issued it
    const int64_t rb = valid ? pf_rb : 0;
    // (a 64-bit min: with only the low halves used the compiler reuses the
    // loaded high half's register at once, a write-after-write wait on the load)
    const int len = CANON ? (valid ? __popc(mask) : 0) : (valid ? (int)min(pf_re - pf_rb, (int64_t)15) : 0);
    if constexpr (HAS_RHS) {  // lanes without a row repeat lane 0's store (always a row)
      if constexpr (CANON && RHS_ADD) pf_rhs = rhs[pf_r];
      const double rv = RHS_ADD ? pf_rhs + g.f_meas * meas : g.f_meas * meas;
      const int64_t r0 = lane_i64(pf_r, 0);
      const double rv0 = lane_f64(rv, 0);
      put<(DIAG & 128) != 0>(&rhs[valid ? pf_r : r0], valid ? rv : rv0);
    }
    // prefix of the row lengths within the x-run (7 lanes), the runs' offsets in the image
    int p = 0;
#pragma unroll
    for (int d = 1; d < kRun; ++d) {
      const int t = __shfl(len, lane - d);
      if (rx - d >= 0) p += t;
    }
    int img0 = 0;  // image offset of this lane's run
#pragma unroll
    for (int q = 0; q < kRun; ++q) {
      const int rl = lane_i32(p + len, kRun * q + kRun - 1);
      if (q < ry) img0 += rl;
    }
    wave_lds_order();  // every lane's accumulator reads before the image overwrites them
    double* img = &acc[b][0][0];
    if constexpr (CANON) {
      // row L's values at [15 L, 15 L + 15) in the caller's column order; its
      // first value and length in the free coordinate buffer of layer z & 1
      int64_t* const rbs = reinterpret_cast<int64_t*>(&cz[NCZ == 1 ? 0 : (z & 1)][0][0]);
      int* const lens = reinterpret_cast<int*>(rbs + 64);
      rbs[lane] = rb;
      lens[lane] = len;
      if (valid) {
#pragma unroll
        for (int o = 0; o < 15; ++o)
          if ((mask >> o) & 1u) {
            const int t = __popc(mask & ((1u << o) - 1u));  // canonical slot (sorted lattice indices)
            img[15 * lane + (int)((pf_slot >> (4 * t)) & 15u)] = v[o];
          }
      }
      wave_lds_order();
      // row by row, consecutive lanes over a row's values; positions past a
      // row's length repeat row 0's first value (always a row), so the store
      // count is fixed
      const int64_t rb0 = rbs[0];
      if constexpr ((DIAG & 512) != 0) {
        // 16 B per lane: pair k of row L = values j, j + 1 with j = min(2k, len - 2)
        // (the last pair overlaps the one before: same values), 8 pairs per row,
        // 7 stores per layer instead of 12; rows without values repeat row 0's
        // first pair
        typedef double d2u __attribute__((ext_vector_type(2), aligned(8)));
#pragma unroll
        for (int i = 0; i < (8 * kRows + 63) / 64; ++i) {
          const int Q = min(64 * i + lane, 8 * kRows - 1);
          const int L = Q >> 3, k = Q & 7;
          const int len = lens[L];
          const bool ok = len >= 2;
          const int j = ok ? min(2 * k, len - 2) : 0;
          const int src = ok ? 15 * L + j : 0;
          *reinterpret_cast<d2u*>(&vals[ok ? rbs[L] + j : rb0]) = d2u{ img[src], img[src + 1] };
        }
      }
      else {
#pragma unroll
        for (int i = 0; i < (15 * kRows + 63) / 64; ++i) {
          const int P = min(64 * i + lane, 15 * kRows - 1);
          const int L = P / 15, j = P - 15 * L;
          const bool ok = j < lens[L];
          put<(DIAG & 128) != 0>(&vals[ok ? rbs[L] + j : rb0], img[ok ? P : 0]);
        }
      }
    }
    else {
    if (valid) {
#pragma unroll
      for (int o = 0; o < 15; ++o)
        if ((mask >> o) & 1u) {
          const int grp = o < 4 ? 0 : (o < 11 ? 1 : 2);
          const uint32_t gmask = grp == 0 ? gm0 : (grp == 1 ? gm1 : gm2);
          const int start = grp == 0 ? s0 : (grp == 1 ? s1 : s2);
          img[img0 + p + start + __popc(gmask & ((1u << o) - 1u))] = v[o];
        }
    }
    wave_lds_order();
    // x-run q: run_len(q) values from image offset img(q) to vals + rb(first row of run q).
    // A fixed count of unpredicated stores: lanes past a run repeat the first
    // value of run 0 (row 0 of the column is always a row: same address, same
    // value), so the next layer's waits on its coordinate loads count past them
    const int64_t dst0 = lane_i64(rb, 0);
    int off = 0;
#pragma unroll
    for (int q = 0; q < kRun; ++q) {
      const int rl = lane_i32(p + len, kRun * q + kRun - 1);
      const int64_t dst = lane_i64(rb, kRun * q);
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // rl <= 7 rows x 15 = 105
        const int t = lane + 64 * h;
        const bool ok = t < rl;
        put<(DIAG & 128) != 0>(&vals[ok ? dst + t : dst0], img[ok ? off + t : 0]);
      }
      off += rl;
    }
    }
    wave_lds_order();
    if constexpr ((kAcc * STRIDE) % 2 == 0) {  // 16-B stores (64-row planes: buffers 16-B aligned)
      double2* const img2 = reinterpret_cast<double2*>(img);
#pragma unroll
      for (int i = 0; i < (kAcc * STRIDE / 2 + 63) / 64; ++i)
        img2[min(64 * i + lane, kAcc * STRIDE / 2 - 1)] = make_double2(0.0, 0.0);
    }
    else {
#pragma unroll
      for (int i = 0; i < (kAcc * STRIDE + 63) / 64; ++i) img[min(64 * i + lane, kAcc * STRIDE - 1)] = 0.0;
    }
    wave_lds_order();
  };

  // ---- cube layer zc: the lane's cube, its 6 tets, 19 edge sums and 8 corner |det| sums
  // CARRY: the top face of the lane's cube (5 edges, 4 corner |det| sums) is
  // the bottom face of its next cube layer, evaluated by the same lane: its
  // sums stay in registers and go into LDS once, with the next cube's
  double ce[5] = { 0.0, 0.0, 0.0, 0.0, 0.0 }, cm[4] = { 0.0, 0.0, 0.0, 0.0 };
  // the corners' accumulator rows for cube layer zc
  auto corner_frame = [&](int zc, uint32_t& inm, int& bb, int& bt) {
    bb = zc & 1;
    bt = (zc + 1) & 1;
    const int rx0 = ci - 1, ry0 = cj - 1;
    const bool zlo = zc >= z0, zhi = zc + 1 < z1;
    const bool xin0 = rx0 >= 0 && cx0 + rx0 < g.npx, xin1 = rx0 + 1 < kRun && cx0 + rx0 + 1 < g.npx;
    const bool yin0 = ry0 >= 0 && cy0 + ry0 < g.npy, yin1 = ry0 + 1 < kRun && cy0 + ry0 + 1 < g.npy;
    inm = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      // (not the lane's cube_in: with the x exchange a corner row takes the
      // neighbour's sums even when this lane's cube is outside the box)
      const bool in = (cbit(c, 0) ? xin1 : xin0) && (cbit(c, 1) ? yin1 : yin0) && (cbit(c, 2) ? zhi : zlo);
      inm |= (uint32_t)in << c;
    }
  };
  // a corner outside the unit adds its zero into the OTHER node layer's
  // buffer at row lane (mod STRIDE): no address shared with the lanes adding
  // real values in the same instruction, none shared among the outside lanes
  // (a clamped row inside the column serialised the same-address adds of
  // neighbouring lanes: 0.73 -> 0.82 ms)
  const int r00 = (ci - 1) + kRun * (cj - 1), rs = lane % STRIDE;
  auto base_at = [&](uint32_t inm, int bb, int bt, int c) {
    const bool in = (inm >> c) & 1u;
    const int buf = (cbit(c, 2) ? bt : bb) ^ (in ? 0 : 1);
    return &acc[buf][0][0] + (in ? r00 + cbit(c, 0) + kRun * cbit(c, 1) : rs);
  };
  // DROWS (V bit 256, 64-row planes): a corner outside the unit (its row
  // index rx or ry outside [0, 6]) adds its REAL sum into a dummy row of its
  // own layer's buffer, rows 49..63, which no store reads: the x-outside
  // lanes (one x edge of the 8 x 8 lanes) at 49 + cj, the other y-outside ones
  // at 57 + rx -- 15 distinct rows for the 15 outside lanes of each corner, so
  // no two lanes of one ds_add_f64 share an address.  No zero selects on the
  // sums, no buffer swap; the rows of node layer z0 - 1 (below the segment,
  // not this unit's) get real sums too, so that buffer is zeroed after the
  // layer below (its next use is node layer z0 + 1).  Rows inside the unit but
  // outside the box take their sums in their own slots and are never stored.
  constexpr bool DROWS = (DIAG & 256) != 0 && STRIDE == 64;
  int row4[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int rx = ci - 1 + (k & 1), ry = cj - 1 + (k >> 1);
    const bool inx = rx >= 0 && rx < kRun, iny = ry >= 0 && ry < kRun;
    row4[k] = (inx && iny) ? rx + kRun * ry : (!inx ? kRows + cj : kRows + 8 + rx);
  }
  auto base_d = [&](int bb, int bt, int c) { return &acc[cbit(c, 2) ? bt : bb][0][0] + row4[c & 3]; };
  // the top face's carried sums into LDS (the box's top node layer: no cube above)
  auto add_top = [&](int zc) {
    uint32_t inm;
    int bb, bt;
    corner_frame(zc, inm, bb, bt);
    auto kept = [&](int c, double x) { return ((inm >> c) & 1u) ? x : 0.0; };
    constexpr int ta[5] = { 4, 4, 4, 5, 6 }, tb[5] = { 5, 6, 7, 7, 7 };
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      if constexpr (DROWS) {
        atomicAdd(base_d(bb, bt, ta[i]) + STRIDE * edge_o(ta[i], tb[i]), ce[i]);
        atomicAdd(base_d(bb, bt, tb[i]) + STRIDE * edge_o(tb[i], ta[i]), ce[i]);
      }
      else {
        atomicAdd(base_at(inm, bb, bt, ta[i]) + STRIDE * edge_o(ta[i], tb[i]), kept(ta[i], ce[i]));
        atomicAdd(base_at(inm, bb, bt, tb[i]) + STRIDE * edge_o(tb[i], ta[i]), kept(tb[i], ce[i]));
      }
    }
#pragma unroll
    for (int c = 4; c < 8; ++c) {
      if constexpr (DROWS)
        atomicAdd(base_d(bb, bt, c) + STRIDE * 7, cm[c - 4]);
      else
        atomicAdd(base_at(inm, bb, bt, c) + STRIDE * 7, kept(c, cm[c - 4]));
    }
  };
  P3 Xc[4];  // the lane's cube's top corners, the next cube layer's bottom ones
  auto prime_corners = [&](int zc) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int q = (ci + cbit(c, 0)) + kCol * (cj + cbit(c, 1));
      const int bz = NCZ == 1 ? 0 : (zc & 1);
      Xc[c] = P3{ cz[bz][0][q], cz[bz][1][q], cz[bz][2][q] };
    }
  };
  auto cubes = [&](int zc) {
    // no branch around the cube: a lane whose cube is outside the box works on
    // its clamped (duplicated) coordinates and adds zeros -- a divergent region
    // here made the compiler drain the next layer's loads (vmcnt(0)) before the
    // arithmetic
    const int bb = zc & 1, bt = (zc + 1) & 1;
    // with CARRY the bottom corners are the previous cube layer's top corners
    // (registers: 12 LDS reads less per layer), the top ones from the staged layer
    P3 X[8];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int q = (ci + cbit(c, 0)) + kCol * (cj + cbit(c, 1));
      const int zb = NCZ == 1 ? 0 : bb, zt = NCZ == 1 ? 0 : bt;
      X[c] = CARRY ? Xc[c] : P3{ cz[zb][0][q], cz[zb][1][q], cz[zb][2][q] };
      X[c + 4] = P3{ cz[zt][0][q], cz[zt][1][q], cz[zt][2][q] };
      if constexpr (CARRY) Xc[c] = X[c + 4];
    }
    double ev[8][8];
    double mv[8];
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      mv[a] = 0.0;
#pragma unroll
      for (int b = 0; b < 8; ++b) ev[a][b] = 0.0;
    }
#pragma unroll
    for (int t = 0; t < ((DIAG & 4) ? 0 : 6); ++t) {
      const int v1 = tet_v(t, 1), v2 = tet_v(t, 2);
      const P3 e1 = psub(X[v1], X[0]), e2 = psub(X[v2], X[0]), e3 = psub(X[7], X[0]);
      P3 k[4];
      k[1] = pcross(e2, e3);
      k[2] = pcross(e3, e1);
      k[3] = pcross(e1, e2);
      k[0] = P3{ -(k[1].x + k[2].x + k[3].x), -(k[1].y + k[2].y + k[3].y), -(k[1].z + k[2].z + k[3].z) };
      // a cube outside the box (clamped, duplicated coordinates) contributes
      // exact zeros: its corners' rows may still take the x-neighbour's sums
      const double meas = cube_in ? fabs(pdot(e1, k[1])) : 0.0;
      const double s = cube_in ? g.s_coef * precip(fmax(meas, 1e-300)) : 0.0;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        mv[tet_v(t, p)] += meas;
#pragma unroll
        for (int q = p + 1; q < 4; ++q) {
          const int a = tet_v(t, p) < tet_v(t, q) ? tet_v(t, p) : tet_v(t, q);
          const int b = tet_v(t, p) < tet_v(t, q) ? tet_v(t, q) : tet_v(t, p);
          ev[a][b] += s * pdot(k[p], k[q]);
        }
      }
    }
    if constexpr (CARRY) {
      // bottom face = the previous cube layer's top face: its carried sums
      ev[0][1] += ce[0];
      ev[0][2] += ce[1];
      ev[0][3] += ce[2];
      ev[1][3] += ce[3];
      ev[2][3] += ce[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) mv[c] += cm[c];
      ce[0] = ev[4][5];
      ce[1] = ev[4][6];
      ce[2] = ev[4][7];
      ce[3] = ev[5][7];
      ce[4] = ev[6][7];
#pragma unroll
      for (int c = 0; c < 4; ++c) cm[c] = mv[c + 4];
    }
    if constexpr (YEX) {
      // the y = 1 face is the y = 0 face of lane + 8's cube: its bottom-layer
      // sums come over first (ds_bpermute; lanes with cj = 7 get their own,
      // their y = 1 corners are outside the unit), so the x exchange below
      // then passes on sums that already hold the diagonal neighbour's
      ev[2][3] += __shfl_down(ev[0][1], 8);
      ev[2][6] += __shfl_down(ev[0][4], 8);
      ev[2][7] += __shfl_down(ev[0][5], 8);
      ev[3][7] += __shfl_down(ev[1][5], 8);
      mv[2] += __shfl_down(mv[0], 8);
      mv[3] += __shfl_down(mv[1], 8);
    }
    if constexpr (XEX) {
      // the x = 1 face of this lane's cube is the x = 0 face of lane + 1's
      // (same 16-lane DPP row; a lane with ci = 7 gets a wrong neighbour but its
      // x = 1 corners are outside the unit): that lane's face sums come over
      // (row_shl:1; zeros from a cube outside the box) and this lane adds
      // both -- 4 edges and 2 corners of the bottom layer (the top face's are
      // carried, and exchanged as the next layer's bottom)
      auto from_next = [&](double x) {
        const long long v = __double_as_longlong(x);
        const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)v, 0x101, 0xf, 0xf, true);
        const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)((unsigned long long)v >> 32), 0x101, 0xf, 0xf, true);
        return __longlong_as_double((long long)(((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo));
      };
      ev[1][3] += from_next(ev[0][2]);
      ev[1][5] += from_next(ev[0][4]);
      ev[1][7] += from_next(ev[0][6]);
      ev[3][7] += from_next(ev[2][6]);
      mv[1] += from_next(mv[0]);
      mv[3] += from_next(mv[2]);
    }
    // each corner's accumulator row: its own when it is a row of this unit,
    // else a zero into the other buffer (base_at); every add runs unpredicated
    uint32_t inm;
    int bb_, bt_;
    corner_frame(zc, inm, bb_, bt_);
    auto kept = [&](int c, double x) { return ((inm >> c) & 1u) ? x : 0.0; };
    double dsum = 0.0;  // DIAG 2
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = a + 1; b < 8; ++b)
        if (is_edge(a, b) && !(CARRY && cbit(a, 2) && cbit(b, 2)) &&
            !(XEX && !cbit(a, 0) && !cbit(b, 0) && !(cbit(a, 2) && cbit(b, 2))) &&
            !(YEX && !cbit(a, 1) && !cbit(b, 1) && !(cbit(a, 2) && cbit(b, 2)))) {
          if constexpr (DIAG & 2) {
            dsum += ev[a][b];
          }
          else if constexpr (DROWS) {
            atomicAdd(base_d(bb_, bt_, a) + STRIDE * edge_o(a, b), ev[a][b]);
            atomicAdd(base_d(bb_, bt_, b) + STRIDE * edge_o(b, a), ev[a][b]);
          }
          else {
            atomicAdd(base_at(inm, bb_, bt_, a) + STRIDE * edge_o(a, b), kept(a, ev[a][b]));
            atomicAdd(base_at(inm, bb_, bt_, b) + STRIDE * edge_o(b, a), kept(b, ev[a][b]));
          }
        }
#pragma unroll
    for (int c = 0; c < 8; ++c)
      if (!(CARRY && cbit(c, 2)) && !(XEX && !cbit(c, 0) && !cbit(c, 2)) && !(YEX && !cbit(c, 1) && !cbit(c, 2))) {
        if constexpr (DIAG & 2)
          dsum += mv[c];
        else if constexpr (DROWS)
          atomicAdd(base_d(bb_, bt_, c) + STRIDE * 7, mv[c]);  // |det| sums
        else
          atomicAdd(base_at(inm, bb_, bt_, c) + STRIDE * 7, kept(c, mv[c]));  // |det| sums
      }
    if constexpr ((DIAG & 2) != 0) atomicAdd(&acc[bb_][0][rs], dsum);
  };

  // ---- walk the cube layers upwards (coordinates staged one layer ahead)
  // the node layers of cube layer zc sit in buffers zc & 1 and (zc + 1) & 1;
  // layer zc + 2's coordinates are loaded at the top of iteration zc and
  // staged at its end (into buffer zc & 1, read for the last time by the
  // cubes): their wait then counts past the flush's stores (vmcnt(N)), and no
  // wait sits at the loop head, where the entry and the back edge would merge
  // into the stricter one
  prefetch_ids(zc_first);
  load_layer(zc_first);
  store_layer(zc_first & 1);
  prefetch_ids(zc_first + 1);
  load_layer(zc_first + 1);
  if constexpr (NCZ == 1) {  // the bottom layer into the corner registers before the top overwrites it
    wave_lds_order();
    prime_corners(zc_first);
    wave_lds_order();
  }
  store_layer((zc_first + 1) & 1);
  wave_lds_order();
  if constexpr (CARRY && NCZ == 2) prime_corners(zc_first);
  int zc = zc_first;
  if (zc < z0) {  // the cube layer below the segment: its top corners only, no flush
    prefetch_ids(zc + 2);
    load_layer(zc + 2);
    wave_lds_order();
    cubes(zc);
    wave_lds_order();
    if constexpr (DROWS) {  // node layer z0 - 1's buffer took real sums: clear it for node layer z0 + 1
      double2* const b2 = reinterpret_cast<double2*>(&acc[zc & 1][0][0]);
#pragma unroll
      for (int i = 0; i < (kAcc * STRIDE / 2 + 63) / 64; ++i)
        b2[min(64 * i + lane, kAcc * STRIDE / 2 - 1)] = make_double2(0.0, 0.0);
      wave_lds_order();
    }
    store_layer(zc & 1);
    ++zc;
  }
  // every layer of the loop completes a node layer of the segment (z0 <= zc
  // <= zc_last < z1): the flush is unconditional, so the offsets' prefetch
  // stays ahead of the cubes
  for (; zc <= zc_last; ++zc) {
    // the offsets of the rows this iteration completes, then the coordinates
    // of layer zc + 2: the flush waits for the offsets only (counted vmcnt)
    prefetch_ids(zc + 2);  // CANON: the next staged layer's caller ids, in flight during the cubes
    prefetch_rows(zc);
    if constexpr ((DIAG & 16) != 0) load_layer(zc + 2);  // before the cubes: their latency hides behind them
    wave_lds_order();
    cubes(zc);
    if constexpr ((DIAG & 16) == 0) load_layer(zc + 2);  // after the cubes: its 12 registers are not live across them
    wave_lds_order();
    flush(zc);
    store_layer(zc & 1);
  }
  if (zc_last + 1 >= z0 && zc_last + 1 < z1) {  // the box's top layer (no cube above)
    prefetch_rows(zc_last + 1);
    if constexpr (CARRY) {
      add_top(zc_last);
      wave_lds_order();
    }
    flush(zc_last + 1);
  }
}

// the staged canonical path's maps, per lattice node i (caller row phys[i]):
// lat[row] = i, and for each position p of the row's columns the Kuhn offset o
// whose value goes there (canonical slot t = the rank of o among the present
// offsets, position = slot[i] >> 4t)
__global__ void k_cube_stage_maps(int64_t n, int npx, int npy, int nzc, const int32_t* __restrict__ phys,
                                  const uint64_t* __restrict__ slot, int32_t* __restrict__ lat,
                                  uint64_t* __restrict__ pinv)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t L = (int64_t)npx * npy;
  const int z = (int)(i / L);
  const int64_t rem = i - (int64_t)z * L;
  const int y = (int)(rem / npx), x = (int)(rem - (int64_t)y * npx);
  uint32_t mask = 0;
  for (int o = 0; o < 15; ++o) {
    const int xx = x + kOffX[o], yy = y + kOffY[o], zz = z + kOffZ[o];
    if (xx >= 0 && yy >= 0 && xx < npx && yy < npy && zz >= 0 && zz <= nzc) mask |= 1u << o;
  }
  const uint64_t sl = slot[i];
  uint64_t w = 0;
  for (int o = 0; o < 15; ++o)
    if ((mask >> o) & 1u) {
      const int t = __popc(mask & ((1u << o) - 1u));
      const int pos = (int)((sl >> (4 * t)) & 15u);
      w |= (uint64_t)o << (4 * pos);
    }
  const int32_t r = phys[i];
  lat[r] = (int32_t)i;
  pinv[r] = w;
}

// the staged canonical path, second pass: caller rows r = 64 w + lane of
// wave w.  Each lane loads its row's lattice line (one aligned 128-B line:
// 8 16-B loads), puts it in LDS, picks its values into the wave's image in
// column order (row r at [rb_r - rb_0, +len)), and the wave stores the image
// -- the 64 rows' values, contiguous in the caller's matrix -- with
// consecutive lanes and 16-B stores: whole lines, where the single-pass
// canonical flush wrote each 120-B row into lines that other units complete
// at other times (WRITE_SIZE 1.77 GB for 1.28 GB)
constexpr int kUnLine = 18;  // LDS doubles per line (16 + 2: 16-B aligned, lanes l and l + 16 share banks only)
// UV: 1 non-temporal line loads, 2 non-temporal value stores -- both by default
// (the lines are read once, the values not by this launch): c2_arrays 1.102 ->
// 1.066 ms (r05bl; 1.094 / 1.075 with one of them); AFEM_UNSTAGE_V=0 / 1 / 2 for A/B
template <bool HAS_RHS, bool RHS_ADD, int UV = 3>
__global__ __launch_bounds__(64) void k_cube_unstage(int64_t n, const int64_t* __restrict__ rp,
                                                      const int32_t* __restrict__ lat,
                                                      const uint64_t* __restrict__ pinv,
                                                      const double* __restrict__ stage, double f_meas,
                                                      double* __restrict__ vals, double* __restrict__ rhs)
{
  __shared__ __align__(16) double line[64 * kUnLine];
  __shared__ __align__(16) double out[64 * 15 + 2];
  const int lane = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * 64;
  const int64_t r = r0 + lane;
  const bool valid = r < n;
  const int64_t rc = valid ? r : n - 1;
  const int64_t rb = rp[rc], re = rp[rc + 1];
  const int64_t li = lat[rc];
  const uint64_t m = pinv[rc];
  typedef double d2a __attribute__((ext_vector_type(2), aligned(16)));
  // load k: lanes 8 j .. 8 j + 7 read row 8 k + j's line, 16 B each (8 whole
  // lines per instruction, not 64 pieces of 64 lines)
  const int part = lane & 7;
  d2a w[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int64_t lk = __shfl((int)li, 8 * k + (lane >> 3));
    if constexpr ((UV & 1) != 0)
      w[k] = __builtin_nontemporal_load(reinterpret_cast<const d2a*>(stage + 16 * lk) + part);
    else
      w[k] = reinterpret_cast<const d2a*>(stage + 16 * lk)[part];
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) reinterpret_cast<d2a*>(line + kUnLine * (8 * k + (lane >> 3)))[part] = w[k];
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if constexpr (HAS_RHS) {
    const double meas = line[kUnLine * lane + 15];
    if (valid) rhs[r] = RHS_ADD ? rhs[r] + f_meas * meas : f_meas * meas;
  }
  const int nv = (int)min((int64_t)64, n - r0);  // rows of this wave
  const int64_t rb0 = rp[r0], re1 = rp[r0 + nv];
  const int a = (int)(rb0 & 1);  // image offset: pairs 16-B aligned in the matrix
  const int len = valid ? (int)(re - rb) : 0;
  const int base = a + (int)(rb - rb0);
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int p = 0; p < 15; ++p)
    if (p < len) out[base + p] = line[kUnLine * lane + (int)((m >> (4 * p)) & 15u)];
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const int total = a + (int)(re1 - rb0);
#pragma unroll
  for (int k = 0; k < (64 * 15 + 2) / 128 + 1; ++k) {
    const int j = 2 * (64 * k + lane);
    if (j < total) {
      double* const g = vals + (rb0 - a + j);
      const bool lo = j >= a, hi = j + 1 < total;
      if (lo && hi) {
        if constexpr ((UV & 2) != 0)
          __builtin_nontemporal_store(d2a{ out[j], out[j + 1] }, reinterpret_cast<d2a*>(g));
        else
          *reinterpret_cast<d2a*>(g) = d2a{ out[j], out[j + 1] };
      }
      else if (lo)
        g[0] = out[j];
      else if (hi)
        g[1] = out[j + 1];
    }
  }
}

}  // namespace

bool assemble_cubes(Bsr& b, double coef, double f, double* rhs, int rhs_add)
{
  const Mesh& m = *b.mesh;
  const StructuredInfo& st = m.st;
  Structure& S = b.s;
  const char* ce = variant("AFEM_ASSEMBLY_CUBES");  // 0: the strip / stencil kernels
  if ((ce && atoi(ce) == 0) || m.nv != 4 || b.nb_dof != 1) return false;
  // a generator box (or z-slab of one), a lattice of Kuhn cubes in a natural
  // numbering (lexicographic in some axis order: the plain instance, with the
  // lattice axes in that order -- the kernel's geometry reads the real
  // coordinates, and the cube's 6 tets do not depend on the axis order), or
  // one in any other numbering (the caller's maps)
  const bool natural = S.cube_natural;
  const bool canon = !natural && S.canon && S.cube_ok;
  if (!canon && !natural && (!st.valid || st.dim != 3 || S.canon || st.lx > 0 || st.ly > 0 || st.n < 1)) return false;
  Ctx& ctx = *m.ctx;
  CubeGeom g{};
  if (canon || natural) {
    const int64_t* Lc = natural ? S.nat_L : S.cube_L;
    g.npx = (int)Lc[0];
    g.npy = (int)Lc[1];
    g.nzc = (int)Lc[2] - 1;
    g.k0 = 0;
    g.k1 = (int)Lc[2];
    g.ghost_lo = g.ghost_hi = -1;
    g.L = Lc[0] * Lc[1];
  }
  else {
    g.npx = g.npy = st.n + 1;
    g.nzc = st.nz;
    g.k0 = st.k0;
    g.k1 = st.k1;
    g.ghost_lo = st.ghost_lo;
    g.ghost_hi = st.ghost_hi;
    g.L = st.L;
    if (g.L != (int64_t)g.npx * g.npy) return false;
  }
  g.n_own_layers = g.k1 - g.k0;
  if (g.n_own_layers <= 0 || g.nzc < 1 || g.npx < 2 || g.npy < 2) return false;
  g.tx = (g.npx + kRun - 1) / kRun;
  g.ty = (g.npy + kRun - 1) / kRun;
  const char* ze = variant("AFEM_CUBES_ZS");
  // z segment: ~n/16 layers (C2 n = 215: 13, C4 n = 463: 29; r04x: zs 12 0.645 ms
  // vs zs 8 0.649 at C2, zs 32 6.38 vs zs 24 6.81 ms at C4)
  g.zs = std::max(1, ze ? atoi(ze) : std::min(48, std::max(8, std::max(g.npx, g.npy) / 16)));
  g.ns = (g.n_own_layers + g.zs - 1) / g.zs;
  g.s_coef = coef / 6.0;
  g.f_meas = f / 24.0;
  const char* fe = variant("AFEM_CUBES_FULL");
  g.full_flush = (fe && atoi(fe) == 0) ? 0 : 1;
  const int64_t n_units = (int64_t)g.tx * g.ty * g.ns;
  AFEM_REQUIRE(n_units < (int64_t(1) << 31), AFEM_ERR_LIMIT, "cube kernel: too many units");
  // accumulator planes of 64 rows (19.3 KB of LDS, 8 waves per CU), or of 49
  // (AFEM_CUBES_STRIDE=49: 15.6 KB, 10 waves -- with the carry it spills: r04y)
  const char* se = variant("AFEM_CUBES_STRIDE");
  const bool s49 = se && atoi(se) == 49;
  // the top face's sums carried in registers to the next cube layer (AFEM_CUBES_CARRY=0: not;
  // r04y C2: 0.605 ms with the carry at 64-row planes, 0.660 without at 49); the x = 1 face's
  // shared with lane + 1 over DPP (AFEM_CUBES_XEX=0: not; needs the carry)
  const char* ke = variant("AFEM_CUBES_CARRY");
  const bool carry = canon || !(ke && atoi(ke) == 0);
  const char* xe = variant("AFEM_CUBES_XEX");
  const bool xex = canon || (carry && !(xe && atoi(xe) == 0));
  // and the y = 1 face's with lane + 8 (AFEM_CUBES_YEX=0: not; needs the x exchange)
  const char* ye = variant("AFEM_CUBES_YEX");
  const bool yex = canon || (xex && !(ye && atoi(ye) == 0));
#define AFEM_CUBES_K(S, C, X, Y, N)                                                                                  \
  (rhs ? (rhs_add ? &k_assemble_cubes<S, C, X, Y, N, true, true> : &k_assemble_cubes<S, C, X, Y, N, true, false>)    \
       : &k_assemble_cubes<S, C, X, Y, N, false, false>)
  const char* de = variant("AFEM_CUBES_V");
  const int diag = de ? atoi(de) : kCubesV;
  // canonical structures: the staged instance (below), or the single-pass one (V without 1024)
  auto* kern = canon ? (rhs ? (rhs_add ? &k_assemble_cubes<64, true, true, true, true, true, true, kCubesV & ~1024>
                                       : &k_assemble_cubes<64, true, true, true, true, true, false, kCubesV & ~1024>)
                            : &k_assemble_cubes<64, true, true, true, true, false, false, kCubesV & ~1024>)
               : carry ? (xex ? (yex ? (s49 ? AFEM_CUBES_K(49, true, true, true, false)
                                            : AFEM_CUBES_K(64, true, true, true, false))
                                     : AFEM_CUBES_K(64, true, true, false, false))
                              : AFEM_CUBES_K(64, true, false, false, false))
                       : (s49 ? AFEM_CUBES_K(49, false, false, false, false) : AFEM_CUBES_K(64, false, false, false, false));
#undef AFEM_CUBES_K
  // AFEM_CUBES_V: another variant of the headline instance (generator boxes and
  // natural lattices, RHS set) or of the canonical one (RHS set)
  if (diag != kCubesV && carry && xex && yex && rhs && !rhs_add) {
    switch (diag) {
#define AFEM_CUBES_D(D)                                                                                              \
  case D:                                                                                                            \
    kern = canon ? &k_assemble_cubes<64, true, true, true, true, true, false, D>                                    \
                 : &k_assemble_cubes<64, true, true, true, false, true, false, D>;                                  \
    break;
      AFEM_CUBES_D(0) AFEM_CUBES_D(112) AFEM_CUBES_D(kCubesV | 1) AFEM_CUBES_D(kCubesV | 4)
      AFEM_CUBES_D(kCubesV | 8) AFEM_CUBES_D(kCubesV | 2) AFEM_CUBES_D(kCubesV & ~512) AFEM_CUBES_D(kCubesV & ~1024)
      AFEM_CUBES_D(kCubesV & ~32)
#undef AFEM_CUBES_D
      default: break;
    }
  }
  CubeCanon cc{ canon ? S.cube_phys.p : nullptr, canon ? S.cube_rb.p : nullptr, canon ? S.cube_slot.p : nullptr,
                nullptr };
  // the canonical path staged (V bit 1024): the cube kernel writes lattice-order
  // lines (no row maps, no RHS), k_cube_unstage moves them into the caller's rows
  // (every lattice node one of this structure's rows, as canonical_lattice builds it)
  const int64_t n_lat = g.L * (int64_t)(g.nzc + 1);
  const bool staged = canon && (diag & 1024) != 0 && n_lat == S.n_rows;
  if (staged) {
    if (S.cube_lat.n != (size_t)n_lat) {
      S.cube_lat.alloc(n_lat);
      S.cube_pinv.alloc(n_lat);
      hipLaunchKernelGGL(k_cube_stage_maps, dim3(grid_for(n_lat, 256)), dim3(256), 0, ctx.stream, n_lat, g.npx, g.npy,
                         g.nzc, S.cube_phys.p, S.cube_slot.p, S.cube_lat.p, S.cube_pinv.p);
      AFEM_LAUNCHED();
    }
    if (b.cube_stage.n != (size_t)(16 * n_lat)) b.cube_stage.alloc(16 * n_lat);
    cc.stage = b.cube_stage.p;
    kern = &k_assemble_cubes<64, true, true, true, true, false, false, kCubesV | 1024>;
    if (diag != kCubesV) {
      switch (diag) {
#define AFEM_CUBES_S(D)                                                                                              \
  case D:                                                                                                            \
    kern = &k_assemble_cubes<64, true, true, true, true, false, false, D>;                                          \
    break;
        AFEM_CUBES_S(kCubesV | 1024 | 1) AFEM_CUBES_S(kCubesV | 1024 | 4)
#undef AFEM_CUBES_S
        default: break;
      }
    }
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)n_units), dim3(64), 0, ctx.stream, g, S.row_ptr.p, m.coords.p, b.values.p,
                     rhs, cc);
  AFEM_LAUNCHED();
  if (staged) {
    const int64_t n = S.n_rows;
    auto* un = rhs ? (rhs_add ? &k_cube_unstage<true, true> : &k_cube_unstage<true, false>)
                   : &k_cube_unstage<false, false>;
    const char* uve = variant("AFEM_UNSTAGE_V");
    const int uv = uve ? atoi(uve) : 3;
    if (rhs && !rhs_add && uv == 0) un = &k_cube_unstage<true, false, 0>;
    if (rhs && !rhs_add && uv == 1) un = &k_cube_unstage<true, false, 1>;
    if (rhs && !rhs_add && uv == 2) un = &k_cube_unstage<true, false, 2>;
    hipLaunchKernelGGL(un, dim3((unsigned)grid_for(n, 64)), dim3(64), 0, ctx.stream, n, S.row_ptr.p, S.cube_lat.p,
                       S.cube_pinv.p, b.cube_stage.p, g.f_meas, b.values.p, rhs);
    AFEM_LAUNCHED();
  }
  b.last_kernel = AFEM_KERNEL_CUBES;
  return true;
}

}  // namespace afem
