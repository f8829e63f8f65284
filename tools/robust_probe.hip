// Probe: HBM -> LDS-DMA throughput of the robust kernels' access pattern
// (K peer rows x RB contiguous bytes per tile, rows 400 MB apart), without
// the sort.  Answers: which row width / blocks per CU / buffering keeps HBM
// busy.  Build: hipcc --offload-arch=gfx950 -O3 -o tools/robust_probe tools/robust_probe.hip
// Run: tools/robust_probe K N   (N coordinates per peer)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define LDS_AS __attribute__((address_space(3)))
#define GLB_AS __attribute__((address_space(1)))
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ void glds16(const float* src, uint8_t LDS_AS* dst) {
  __builtin_amdgcn_global_load_lds((GLB_AS void*)(const_cast<float*>(src)), (LDS_AS void*)dst, 16, 0, 0);
}

// W waves per block, tile = RB bytes of each of K rows; BUF LDS buffers.
// SPIN: VALU cycles of fake work per tile (emulates the sort).
template <int RB, int W, int K, int BUF>
__global__ __launch_bounds__(64 * W) void probe(const float* const* peers, int64_t ntiles, int spin,
                                                float* sink) {
  constexpr int TB = RB / 4;               // coordinates per tile
  constexpr int LPR = RB / 16;             // lanes per row
  constexpr int RPC = 1024 / RB;           // rows per DMA instruction
  constexpr int NCH = K / RPC;             // instructions per tile
  constexpr int NCHW = NCH / W;
  __shared__ __attribute__((aligned(16))) uint8_t lds_raw[BUF * K * RB];
  uint8_t LDS_AS* lds = (uint8_t LDS_AS*)lds_raw;
  const int wi = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const float* rp[NCHW];
#pragma unroll
  for (int m = 0; m < NCHW; ++m) rp[m] = peers[(wi * NCHW + m) * RPC + lane / LPR];
  const int64_t nb = gridDim.x;
  int64_t t = blockIdx.x;
  if ((nb & 7) == 0) t = (blockIdx.x & 7) * (nb >> 3) + (blockIdx.x >> 3);
  float acc = 0.f;
  auto issue = [&](int64_t tt, int b) {
    const int64_t off = tt * TB + 4 * (lane % LPR);
#pragma unroll
    for (int m = 0; m < NCHW; ++m) glds16(rp[m] + off, lds + b * K * RB + (wi * NCHW + m) * 1024);
  };
  int b = 0;
  if (t < ntiles) issue(t, 0);
  if (BUF == 2 && t + nb < ntiles) issue(t + nb, 1);
  for (; t < ntiles; t += nb) {
    if (BUF == 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NCHW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    acc += ((const float LDS_AS*)(lds + b * K * RB))[threadIdx.x];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int64_t tn = t + BUF * nb;
    if (tn < ntiles) issue(tn, b);
    for (int s = 0; s < spin; ++s) acc = acc * 1.0000001f + 1e-7f;
    b = BUF == 2 ? 1 - b : 0;
  }
  if (acc == 12345.f) sink[0] = acc;
}

template <int RB, int W, int K, int BUF>
static void run(const char* tag, const float* const* d_peers, int64_t n, int spin, float* sink) {
  auto kern = probe<RB, W, K, BUF>;
  int per_cu = 0, cus = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kern), 64 * W, 0));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int64_t ntiles = n / (RB / 4);
  const int grid = cus * per_cu;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * W), 0, 0, d_peers, ntiles, spin, sink);
  CHECK(hipEventRecord(e0));
  const int reps = 3;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * W), 0, 0, d_peers, ntiles, spin, sink);
  CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
  float ms = 0; CHECK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
  const double bytes = 4.0 * K * ntiles * (RB / 4);
  printf("%-28s RB=%4d W=%d BUF=%d blocks/CU=%d spin=%5d  %8.3f ms  %7.1f GB/s  (%.1f%% of 8 TB/s)\n", tag, RB, W, BUF,
         per_cu, spin, ms, bytes / ms / 1e6, bytes / ms / 1e6 / 80.0);
}

int main(int argc, char** argv) {
  constexpr int K = 256;
  const int64_t n = argc > 1 ? atoll(argv[1]) : 50000000;
  float* slab;
  CHECK(hipMalloc(&slab, sizeof(float) * K * n));
  CHECK(hipMemset(slab, 0, sizeof(float) * K * n));
  const float* h[K];
  for (int k = 0; k < K; ++k) h[k] = slab + (int64_t)k * n;
  const float** d_peers;
  CHECK(hipMalloc(&d_peers, sizeof(h)));
  CHECK(hipMemcpy(d_peers, h, sizeof(h), hipMemcpyHostToDevice));
  float* sink; CHECK(hipMalloc(&sink, 4));
  for (int spin : {0, 1000, 2000}) {
    run<64, 1, K, 1>("64B rows, 1 wave", d_peers, n, spin, sink);
    run<128, 2, K, 1>("128B rows, 2 waves", d_peers, n, spin, sink);
    run<256, 4, K, 1>("256B rows, 4 waves", d_peers, n, spin, sink);
    run<256, 4, K, 2>("256B rows, 4 waves, 2 buf", d_peers, n, spin, sink);
    run<512, 4, K, 1>("512B rows, 4 waves", d_peers, n, spin, sink);
    run<512, 8, K, 1>("512B rows, 8 waves", d_peers, n, spin, sink);
  }
  return 0;
}
