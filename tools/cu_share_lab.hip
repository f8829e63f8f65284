// Lab (round 6, VERDICT r05 missing #1 / DESIGN §7): does a collective's
// kernel get CUs while the FedAvg split kernel runs?  One GPU, two streams:
// the product's p2p_aggregate_ex_f32 (FedAvg, K peers x n) on stream A and,
// launched right behind it on stream B, a stand-in for RCCL's all-gather
// kernel with its resource shape (ncclDevKernel_Generic on gfx950: 512
// threads, 36.8 KiB of LDS -- too much LDS to sit beside a 128-KiB split
// block on a 160-KiB CU) copying the bytes a cfg3 plane's all-gather writes
// at N = 8.  Device wall clock (s_memrealtime, 100 MHz) stamps: the split
// launch's start and end (marker kernels around it on stream A), the
// stand-in's first block start and last block end.  Hints: 0 (the tile
// queue's persistent grid for K <= 128) and P2P_HINT_SHARE_CUS (one block
// per tile).  Measurement tool, not product.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -o tools/cu_share_lab tools/cu_share_lab.hip \
//          -L p2pdl_amd -lp2pdl_hip -Wl,-rpath,'$ORIGIN/../p2pdl_amd'
// Run: tools/cu_share_lab K n copy_bytes blocks reps
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "p2pdl.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

// stamps[0] = first block start (min), stamps[1] = last block end (max)
__global__ __launch_bounds__(512) void standin_copy(const float4* __restrict__ src, float4* __restrict__ dst, long n4,
                                                    unsigned long long* stamps) {
  __shared__ float4 lds[36 * 1024 / 16 + 48];  // 36.8 KiB, as ncclDevKernel_Generic
  const uint64_t t0 = now();
  if (threadIdx.x == 0) atomicMin(&stamps[0], (unsigned long long)t0);
  for (long i = blockIdx.x * 512L + threadIdx.x; i < n4; i += (long)gridDim.x * 512) {
    float4 v = src[i];
    lds[threadIdx.x] = v;  // staged through LDS like a collective's FIFO (keeps the allocation live)
    dst[i] = lds[threadIdx.x];
  }
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(&stamps[1], (unsigned long long)now());
}

__global__ void marker(unsigned long long* slot) {
  if (threadIdx.x == 0) *slot = now();
}

__global__ void init(float* a, long n, uint32_t salt) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    a[i] = (float)(((i ^ salt) * 2654435761u) & 1023) * (1.0f / 1024) - 0.5f;
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 64;
  const long n = argc > 2 ? atol(argv[2]) : 100007936L;
  const long copy_bytes = argc > 3 ? atol(argv[3]) : 469762048L;  // 7/8 of 16.7M x 8 ranks x 4 B
  const int blocks = argc > 4 ? atoi(argv[4]) : 32;
  const int reps = argc > 5 ? atoi(argv[5]) : 5;
  float *slab, *w, *csrc, *cdst;
  CHECK(hipMalloc(&slab, 4L * K * n)); CHECK(hipMalloc(&w, 4 * n));
  CHECK(hipMalloc(&csrc, copy_bytes)); CHECK(hipMalloc(&cdst, copy_bytes));
  hipLaunchKernelGGL(init, dim3(8192), dim3(256), 0, 0, slab, (long)K * n, 7u);
  hipLaunchKernelGGL(init, dim3(8192), dim3(256), 0, 0, w, n, 99u);
  hipLaunchKernelGGL(init, dim3(8192), dim3(256), 0, 0, csrc, copy_bytes / 4, 5u);
  std::vector<const float*> hp(K);
  for (int k = 0; k < K; ++k) hp[k] = slab + (long)k * n;
  const float** dp; CHECK(hipMalloc(&dp, sizeof(void*) * K));
  CHECK(hipMemcpy(dp, hp.data(), sizeof(void*) * K, hipMemcpyHostToDevice));
  unsigned long long* st; CHECK(hipMalloc(&st, 64));
  hipStream_t a, b;
  CHECK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking)); CHECK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  CHECK(hipDeviceSynchronize());
  const long n4 = copy_bytes / 16;
  auto copy_alone = [&]() {
    unsigned long long h[2] = {~0ull, 0ull};
    CHECK(hipMemcpy(st, h, 16, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(standin_copy, dim3(blocks), dim3(512), 0, b, (const float4*)csrc, (float4*)cdst, n4, st);
    CHECK(hipStreamSynchronize(b));
    CHECK(hipMemcpy(h, st, 16, hipMemcpyDeviceToHost));
    return (h[1] - h[0]) / 100.0;  // us (100 MHz)
  };
  printf("K=%d n=%ld, stand-in all-gather kernel: %d blocks x 512 threads, 36.8 KiB LDS, %.0f MB\n", K, n, blocks,
         copy_bytes / 1e6);
  for (int r = 0; r < 2; ++r) copy_alone();
  printf("stand-in alone: %.1f us\n", copy_alone());
  for (int hint = 0; hint <= 1; ++hint) {
    std::vector<double> split_us, start_lag, end_lag;
    for (int r = 0; r < reps + 1; ++r) {
      unsigned long long h[6] = {~0ull, 0ull, 0, 0, 0, 0};
      CHECK(hipMemcpy(st, h, 48, hipMemcpyHostToDevice));
      CHECK(hipDeviceSynchronize());
      hipLaunchKernelGGL(marker, dim3(1), dim3(64), 0, a, st + 2);
      int32_t rc = p2p_aggregate_ex_f32(dp, K, n, P2P_RULE_FEDAVG, 0, 0.1f, w, nullptr, hint ? P2P_HINT_SHARE_CUS : 0, a);
      if (rc != P2P_OK) { printf("p2p_aggregate_ex_f32: %s\n", p2p_strerror(rc)); return 1; }
      hipLaunchKernelGGL(marker, dim3(1), dim3(64), 0, a, st + 3);
      hipLaunchKernelGGL(standin_copy, dim3(blocks), dim3(512), 0, b, (const float4*)csrc, (float4*)cdst, n4, st);
      CHECK(hipDeviceSynchronize());
      CHECK(hipMemcpy(h, st, 48, hipMemcpyDeviceToHost));
      if (r == 0) continue;  // warm-up
      split_us.push_back((h[3] - h[2]) / 100.0);
      start_lag.push_back(((double)h[0] - (double)h[2]) / 100.0);  // stand-in's first block after the split's start
      end_lag.push_back(((double)h[1] - (double)h[3]) / 100.0);    // stand-in's end after the split's end
    }
    std::sort(split_us.begin(), split_us.end());
    std::sort(start_lag.begin(), start_lag.end());
    std::sort(end_lag.begin(), end_lag.end());
    const size_t m = split_us.size() / 2;
    printf("hint %-16s split launch %8.1f us | stand-in first block %+9.1f us after the split's start, "
           "ends %+9.1f us after its end (medians of %d)\n",
           hint ? "SHARE_CUS" : "0 (queue<=128)", split_us[m], start_lag[m], end_lag[m], reps);
  }
  return 0;
}
