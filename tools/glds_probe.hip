// LDS-DMA probe: where does global_load_lds_dwordx3 put lane l's 12 bytes?
// (one wave; LDS pre-filled with a marker; lane l loads src[3l .. 3l+2] as 3 u32)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void k_probe(const uint32_t* __restrict__ src, uint32_t* __restrict__ out, int mode)
{
  extern __shared__ __align__(16) unsigned char smem[];
  uint32_t* l = reinterpret_cast<uint32_t*>(smem);
  const int lane = threadIdx.x;
  for (int i = lane; i < 1024; i += 64) l[i] = 0xDEADBEEFu;
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)smem;
  const void* g = src + 3 * lane;
  uint32_t keep;
  if (mode == 0)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx3 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(base) : "memory");
  else
    __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)smem, 12, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  for (int i = lane; i < 1024; i += 64) out[i] = l[i];
}

int main()
{
  std::vector<uint32_t> h(4096);
  for (int i = 0; i < 4096; ++i) h[i] = 1000000u + i;
  uint32_t *d_src, *d_out;
  hipMalloc(&d_src, 4096 * 4);
  hipMalloc(&d_out, 1024 * 4);
  hipMemcpy(d_src, h.data(), 4096 * 4, hipMemcpyHostToDevice);
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 4096, 0, d_src, d_out, mode);
    std::vector<uint32_t> o(1024);
    hipMemcpy(o.data(), d_out, 1024 * 4, hipMemcpyDeviceToHost);
    printf("mode %d:", mode);
    int bad = 0;
    for (int i = 0; i < 192; ++i)
      if (o[i] != 1000000u + i) ++bad;
    printf(" mismatches in the first 192 dwords vs lane*12 layout: %d\n", bad);
    for (int i = 0; i < 200; ++i) printf("%s%u", i % 16 ? " " : "\n  ", o[i] >= 1000000u && o[i] < 1100000u ? o[i] - 1000000u : 99999u);
    printf("\n");
  }
  return 0;
}
