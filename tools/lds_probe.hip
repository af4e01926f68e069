// LDS micro-probe (diagnostic, not part of libafem): cost and bank conflicts
// of the access patterns of the strip assembly kernel on gfx950.
//   build: hipcc -O3 --offload-arch=gfx950 tools/lds_probe.hip -o tools/lds_probe
//   run:   rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS --kernel-trace --stats -- tools/lds_probe
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 4096;

// lane -> (i,j,k) in a 4x4x4 brick; node of step offset (dx,dy,dz); index in a
// 6x6x6 box (the sorted slice node list of a full brick, approximately)
__device__ __forceinline__ int box_u(int lane, int dx, int dy, int dz)
{
  const int i = lane & 3, j = (lane >> 2) & 3, k = lane >> 4;
  return (i + dx + 1) + 6 * (j + dy + 1) + 36 * (k + dz + 1);
}

__global__ __launch_bounds__(64) void k_add_slot_lane(double* out, int s0)
{
  __shared__ double acc[16 * 64];
  const int lane = threadIdx.x;
  for (int q = lane; q < 16 * 64; q += 64) acc[q] = 0.0;
  __builtin_amdgcn_wave_barrier();
  double v = lane * 1e-3;
  for (int it = 0; it < ITERS; ++it) {
    const int slot = (it * 7 + s0) & 15;  // wave-uniform slot
    atomicAdd(&acc[slot * 64 + lane], v);
    v += 1e-9;
  }
  __builtin_amdgcn_wave_barrier();
  out[blockIdx.x * 64 + lane] = acc[lane];
}

template <int S>
__global__ __launch_bounds__(64) void k_add_lane_major(double* out, int s0)
{
  __shared__ double acc[64 * S];
  const int lane = threadIdx.x;
  for (int q = lane; q < 64 * S; q += 64) acc[q] = 0.0;
  __builtin_amdgcn_wave_barrier();
  double v = lane * 1e-3;
  for (int it = 0; it < ITERS; ++it) {
    const int slot = (it * 7 + s0) & 15;
    atomicAdd(&acc[lane * S + slot], v);
    v += 1e-9;
  }
  __builtin_amdgcn_wave_barrier();
  out[blockIdx.x * 64 + lane] = acc[lane * S];
}

// AoS coordinates, 24 B per node (x,y,z adjacent: ds_read2_b64 + ds_read_b64)
__global__ __launch_bounds__(64) void k_read_aos(double* out, int s0)
{
  __shared__ double c[3 * 256];
  const int lane = threadIdx.x;
  for (int q = lane; q < 3 * 256; q += 64) c[q] = q * 0.5;
  __builtin_amdgcn_wave_barrier();
  double acc = 0.0;
  for (int it = 0; it < ITERS; ++it) {
    const int o = (it + s0) % 14;  // one of the 14 Kuhn neighbour offsets
    const int dx = (o % 3) - 1, dy = ((o / 3) % 3) - 1, dz = (o / 9) - 1;
    const int u = box_u(lane, dx, dy, dz);
    acc += c[3 * u] + c[3 * u + 1] * 1.5 + c[3 * u + 2] * 2.5;
  }
  out[blockIdx.x * 64 + lane] = acc;
}

// SoA coordinates with an odd stride of 257 doubles (three ds_read_b64 at immediate offsets)
__global__ __launch_bounds__(64) void k_read_soa(double* out, int s0)
{
  __shared__ double c[3 * 257];
  const int lane = threadIdx.x;
  for (int q = lane; q < 3 * 257; q += 64) c[q] = q * 0.5;
  __builtin_amdgcn_wave_barrier();
  double acc = 0.0;
  for (int it = 0; it < ITERS; ++it) {
    const int o = (it + s0) % 14;
    const int dx = (o % 3) - 1, dy = ((o / 3) % 3) - 1, dz = (o / 9) - 1;
    const int u = box_u(lane, dx, dy, dz);
    acc += c[u] + c[257 + u] * 1.5 + c[514 + u] * 2.5;
  }
  out[blockIdx.x * 64 + lane] = acc;
}

// synthetic index patterns (the index passes through an empty asm so the
// loads stay in the loop): MODE 0 u = lane; 1 u = 16*(lane&15) + (lane>>4)
// (16 lanes on one bank under the 4x16-group model); 2 u = lane + 16*(lane>>4)
// (groups 0-15 / 16-31 overlapping mod 32); 3 u = 2*lane; 4 u = lane ^ 16
template <int MODE>
__global__ __launch_bounds__(64) void k_read_pat(double* out, int s0)
{
  __shared__ double c[3 * 256];
  const int lane = threadIdx.x;
  for (int q = lane; q < 3 * 256; q += 64) c[q] = q * 0.5;
  __builtin_amdgcn_wave_barrier();
  double acc = 0.0;
  for (int it = 0; it < ITERS; ++it) {
    int u;
    if (MODE == 0) u = lane;
    else if (MODE == 1) u = 16 * (lane & 15) + (lane >> 4);
    else if (MODE == 2) u = (lane & 15) + 32 * (lane >> 4);
    else if (MODE == 3) u = 2 * lane;
    else u = lane ^ 16;
    asm volatile("" : "+v"(u));
    acc += c[3 * u] + c[3 * u + 1] * 1.5 + c[3 * u + 2] * 2.5;
  }
  out[blockIdx.x * 64 + lane] = acc;
}

// x/y only (one ds_read2_b64 per iteration) and z only (one ds_read_b64), box pattern
template <int WHICH>
__global__ __launch_bounds__(64) void k_read_part(double* out, int s0)
{
  __shared__ double c[3 * 256];
  const int lane = threadIdx.x;
  for (int q = lane; q < 3 * 256; q += 64) c[q] = q * 0.5;
  __builtin_amdgcn_wave_barrier();
  double acc = 0.0;
  for (int it = 0; it < ITERS; ++it) {
    const int o = (it + s0) % 14;
    const int dx = (o % 3) - 1, dy = ((o / 3) % 3) - 1, dz = (o / 9) - 1;
    int u = box_u(lane, dx, dy, dz);
    asm volatile("" : "+v"(u));
    if (WHICH == 0) acc += c[3 * u] + c[3 * u + 1] * 1.5;
    else acc += c[3 * u + 2] * 2.5;
  }
  out[blockIdx.x * 64 + lane] = acc;
}

int main()
{
  double* d;
  const int blocks = 4096;
  hipMalloc(&d, sizeof(double) * 64 * blocks);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto run = [&](const char* name, auto kern) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, d, rep);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      if (rep) printf("%-24s %8.3f ms  %.2f ns per wave-iteration\n", name, ms, 1e6 * ms / ((double)blocks * ITERS / 1024.0));
    }
  };
  run("add [slot][lane]", k_add_slot_lane);
  run("add [lane][17]", k_add_lane_major<17>);
  run("add [lane][16]", k_add_lane_major<16>);
  run("read AoS 24B", k_read_aos);
  run("read SoA 257", k_read_soa);
  run("read pat u=lane", k_read_pat<0>);
  run("read pat 16-way", k_read_pat<1>);
  run("read pat halves", k_read_pat<2>);
  run("read pat 2lane", k_read_pat<3>);
  run("read pat lane^16", k_read_pat<4>);
  run("read2 xy only", k_read_part<0>);
  run("read z only", k_read_part<1>);
  hipFree(d);
  return 0;
}
