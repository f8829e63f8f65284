// Probe: HBM read rate of LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave
// instruction, no VGPR write-back) against 16-B nontemporal loads into VGPRs,
// over a 16 GB buffer (far past the 256 MiB Infinity Cache).  Decides whether
// a FedAvg that stages peer rows through LDS could beat the VGPR-load kernel
// (fedavg.hip, 95-96% of the VGPR read roof).  Measurement tool, not product.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/dma_roof tools/dma_roof.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));

// VGPR roof: grid-stride nontemporal float4 loads, UN in flight per lane.
template <int UN>
__global__ __launch_bounds__(256) void vgpr_roof(const f4* __restrict__ a, long n4, float* sink) {
  f4 s = {0, 0, 0, 0};
  const long stride = (long)gridDim.x * 256;
  long i = blockIdx.x * 256L + threadIdx.x;
  for (; i + (UN - 1) * stride < n4; i += UN * stride) {
    f4 x[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) x[u] = __builtin_nontemporal_load(a + i + u * stride);
#pragma unroll
    for (int u = 0; u < UN; ++u) s += x[u];
  }
  if (s.x == 1234.5f) sink[0] = s.y;
}

// DMA roof: every wave streams its own contiguous chunk of 1 KiB pieces into
// a private LDS ring of D pieces, keeping at most D in flight (s_waitcnt
// vmcnt).  AUX: cache policy bits (2 = nt).
template <int D, int WAVES, int AUX>
__global__ __launch_bounds__(64 * WAVES) void dma_roof(const float* __restrict__ a, long pieces_per_wave, float* sink) {
  __shared__ __attribute__((aligned(16))) float ring[WAVES][D][256];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long gw = (long)blockIdx.x * WAVES + wv;
  const float* src = a + gw * pieces_per_wave * 256 + lane * 4;
  for (long p = 0; p < pieces_per_wave; ++p) {
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src + p * 256),
                                     (__attribute__((address_space(3))) void*)&ring[wv][p % D][0], 16, 0, AUX);
    if (p >= D - 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D - 1) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (ring[wv][0][lane] == 1234.5f) sink[0] = 1.f;
}

__global__ void init(float* a, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    a[i] = (float)((i * 2654435761u) & 1023) * (1.0f / 1024);
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 4L << 30;  // floats (16 GiB)
  float* a; float* sink;
  CHECK(hipMalloc(&a, n * 4)); CHECK(hipMalloc(&sink, 64));
  hipLaunchKernelGGL(init, dim3(8192), dim3(256), 0, 0, a, n);
  CHECK(hipDeviceSynchronize());
  int cus = 0; CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  struct R { const char* name; void (*fn)(const float*, long, float*, int); };
  static int CUS; CUS = cus;
#define DMA(NAME, D, W, AUX, BPC) {NAME, [](const float* a, long n, float* s, int) { \
    const long waves = (long)CUS * BPC * W; const long ppw = n / 256 / waves; \
    hipLaunchKernelGGL((dma_roof<D, W, AUX>), dim3(CUS * BPC), dim3(64 * W), 0, 0, a, ppw, s); }}
#define VG(NAME, UN, GRID) {NAME, [](const float* a, long n, float* s, int) { \
    hipLaunchKernelGGL((vgpr_roof<UN>), dim3(GRID), dim3(256), 0, 0, (const f4*)a, n / 4, s); }}
  std::vector<R> rs = {
      VG("vgpr nt u1 g8192", 1, 8192), VG("vgpr nt u4 g8192", 4, 8192), VG("vgpr nt u8 g4096", 8, 4096),
      VG("vgpr nt u8 g2048", 8, 2048),
      DMA("dma nt D8 W4 x2/CU", 8, 4, 2, 2), DMA("dma nt D16 W4 x2/CU", 16, 4, 2, 2),
      DMA("dma nt D16 W8 x1/CU", 16, 8, 2, 1), DMA("dma nt D32 W4 x1/CU", 32, 4, 2, 1),
      DMA("dma nt D8 W16 x1/CU", 8, 16, 2, 1), DMA("dma def D16 W4 x2/CU", 16, 4, 0, 2),
      DMA("dma nt D4 W16 x2/CU", 4, 16, 2, 2), DMA("dma nt D32 W2 x4/CU", 32, 2, 2, 4),
  };
  std::vector<std::vector<float>> ms(rs.size());
  for (int rep = 0; rep < 5; ++rep)
    for (size_t r = 0; r < rs.size(); ++r) {
      rs[r].fn(a, n, sink, 0);
      CHECK(hipEventRecord(e0));
      rs[r].fn(a, n, sink, 0);
      CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
      float t; CHECK(hipEventElapsedTime(&t, e0, e1));
      ms[r].push_back(t);
    }
  for (size_t r = 0; r < rs.size(); ++r) {
    std::sort(ms[r].begin(), ms[r].end());
    const float t = ms[r][ms[r].size() / 2];
    printf("%-24s median %8.3f ms  %7.1f GB/s  (%.1f%% of 8 TB/s)  best %.1f GB/s\n", rs[r].name, t, n * 4.0 / (t * 1e-3) / 1e9,
           n * 4.0 / (t * 1e-3) / 8e12 * 100, n * 4.0 / (ms[r][0] * 1e-3) / 1e9);
  }
  return 0;
}
