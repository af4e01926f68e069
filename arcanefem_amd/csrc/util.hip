// Device utilities: error plumbing and a 3-phase exclusive scan (int -> int64).
// The scan is used only by the one-time structure build (row offsets,
// node->cell offsets, incidence-slice offsets), not by the timed assembly.
#include "afem_internal.hpp"

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <set>
#include <string>

namespace afem {

// Kernel-variant knobs (diagnostics and A/B measurements): an
// explicit override (afem_set_variant) wins, else the process environment as
// it was the first time the knob was looked up; unset = the default variant.
namespace {
struct Variants {
  std::mutex mu;
  std::map<std::string, std::string> set;          // afem_set_variant
  std::map<std::string, std::pair<bool, std::string>> env;  // first lookup of the environment
  // every value ever returned, interned: a returned pointer stays valid after a
  // later afem_set_variant replaces or clears the knob (set nodes never move)
  std::set<std::string> pool;
};
Variants& variants()
{
  static Variants v;
  return v;
}
}  // namespace

const char* variant(const char* name)
{
  Variants& v = variants();
  std::lock_guard<std::mutex> g(v.mu);
  auto it = v.set.find(name);
  if (it != v.set.end()) return v.pool.insert(it->second).first->c_str();
  auto e = v.env.find(name);
  if (e == v.env.end()) {
    const char* x = getenv(name);
    e = v.env.emplace(name, std::make_pair(x != nullptr, std::string(x ? x : ""))).first;
  }
  return e->second.first ? e->second.second.c_str() : nullptr;
}

void set_variant(const char* name, const char* value)
{
  Variants& v = variants();
  std::lock_guard<std::mutex> g(v.mu);
  if (value)
    v.set[name] = value;
  else
    v.set.erase(name);
}

void throw_hip(hipError_t e, const char* expr, const char* file, int line)
{
  char buf[512];
  snprintf(buf, sizeof(buf), "%s failed: %s (%s:%d)", expr, hipGetErrorString(e), file, line);
  throw Error(AFEM_ERR_HIP, buf);
}

namespace {

constexpr int kScanThreads = 256;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanThreads * kScanItems;

__device__ __forceinline__ int64_t wave_inclusive_scan(int64_t v)
{
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int64_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

// Block-wide exclusive scan of one value per thread; returns the exclusive
// prefix and the block total through *total.
__device__ __forceinline__ int64_t block_exclusive_scan(int64_t v, int64_t* total)
{
  __shared__ int64_t wsum[kScanThreads / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t inc = wave_inclusive_scan(v);
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  int64_t woff = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kScanThreads / 64; ++w) {
    int64_t s = wsum[w];
    if (w < wid) woff += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return woff + inc - v;
}

template <class In>
__global__ __launch_bounds__(kScanThreads) void k_tile_sums(const In* __restrict__ in, int64_t n, int64_t* __restrict__ sums)
{
  const int64_t base = (int64_t)blockIdx.x * kScanTile;
  int64_t s = 0;
#pragma unroll
  for (int it = 0; it < kScanItems; ++it) {
    int64_t i = base + (int64_t)it * kScanThreads + threadIdx.x;
    if (i < n) s += (int64_t)in[i];
  }
  int64_t tot;
  (void)block_exclusive_scan(s, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

template <class In>
__global__ __launch_bounds__(kScanThreads) void k_tile_scan(const In* __restrict__ in, int64_t n,
                                                            const int64_t* __restrict__ offsets,
                                                            int64_t* __restrict__ out)
{
  const int64_t base = (int64_t)blockIdx.x * kScanTile;
  // each thread scans kScanItems CONSECUTIVE elements
  int64_t v[kScanItems];
  int64_t s = 0;
  const int64_t tb = base + (int64_t)threadIdx.x * kScanItems;
#pragma unroll
  for (int it = 0; it < kScanItems; ++it) {
    int64_t i = tb + it;
    v[it] = (i < n) ? (int64_t)in[i] : 0;
    s += v[it];
  }
  int64_t tot;
  int64_t pre = block_exclusive_scan(s, &tot) + offsets[blockIdx.x];
#pragma unroll
  for (int it = 0; it < kScanItems; ++it) {
    int64_t i = tb + it;
    if (i < n) out[i] = pre;
    pre += v[it];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == kScanThreads - 1) out[n] = pre;
}

template <class In>
void scan_impl(Ctx& ctx, const In* in, int64_t* out, int64_t n)
{
  // out has n+1 entries; out[n] = total
  if (n == 0) {
    AFEM_HIP(hipMemsetAsync(out, 0, sizeof(int64_t), ctx.stream));
    return;
  }
  int64_t nt = (n + kScanTile - 1) / kScanTile;
  DevBuf<int64_t> sums, offs;
  sums.alloc(nt);
  offs.alloc(nt + 1);
  hipLaunchKernelGGL(k_tile_sums<In>, dim3((unsigned)nt), dim3(kScanThreads), 0, ctx.stream, in, n, sums.p);
  AFEM_LAUNCHED();
  if (nt == 1) {
    AFEM_HIP(hipMemsetAsync(offs.p, 0, sizeof(int64_t), ctx.stream));
  }
  else {
    scan_impl<int64_t>(ctx, sums.p, offs.p, nt);
  }
  hipLaunchKernelGGL(k_tile_scan<In>, dim3((unsigned)nt), dim3(kScanThreads), 0, ctx.stream, in, n, offs.p, out);
  AFEM_LAUNCHED();
  // temporaries are freed at scope exit: make sure the kernels are done
  ctx.sync();
}

__global__ void k_minmax_i32(const int32_t* __restrict__ a, int64_t n, int* __restrict__ out)
{
  int lo = INT32_MAX, hi = INT32_MIN;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    lo = min(lo, a[i]);
    hi = max(hi, a[i]);
  }
  for (int d = 32; d > 0; d >>= 1) {
    lo = min(lo, __shfl_xor(lo, d, 64));
    hi = max(hi, __shfl_xor(hi, d, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(out, lo);
    atomicMax(out + 1, hi);
  }
}

}  // namespace

void device_minmax_i32(Ctx& ctx, const int32_t* a, int64_t n, int32_t* lo, int32_t* hi)
{
  *lo = 0;
  *hi = 0;
  if (n <= 0) return;
  DevBuf<int> d;
  d.alloc(2);
  const int init[2] = { INT32_MAX, INT32_MIN };
  AFEM_HIP(hipMemcpyAsync(d.p, init, sizeof(init), hipMemcpyHostToDevice, ctx.stream));
  const unsigned nb = (unsigned)std::min<int64_t>(1024, (n + 255) / 256);
  hipLaunchKernelGGL(k_minmax_i32, dim3(nb), dim3(256), 0, ctx.stream, a, n, d.p);
  AFEM_LAUNCHED();
  int h[2];
  AFEM_HIP(hipMemcpyAsync(h, d.p, sizeof(h), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  *lo = h[0];
  *hi = h[1];
}

void exclusive_scan_i64(Ctx& ctx, const int64_t* in, int64_t* out, int64_t n, DevBuf<int64_t>*)
{
  scan_impl<int64_t>(ctx, in, out, n);
}

void exclusive_scan_i32_to_i64(Ctx& ctx, const int32_t* in, int64_t* out, int64_t n)
{
  scan_impl<int32_t>(ctx, in, out, n);
}

int64_t read_i64(Ctx& ctx, const int64_t* d)
{
  int64_t v = 0;
  AFEM_HIP(hipMemcpyAsync(&v, d, sizeof(int64_t), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  return v;
}

}  // namespace afem
