// Probe: VALU throughput of the robust kernels' register networks (no memory).
// Each lane repeatedly sorts / merges 64 keys in VGPRs; occupancy is pinned
// with dynamic LDS (waves per CU).  Reports VALU instructions per wave-tile and
// achieved ns per wave-tile.
// Build: hipcc --offload-arch=gfx950 -O3 -I p2pdl_amd/csrc -o tools/sort_probe tools/sort_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

// Packed 16-bit keys (two coordinates per VGPR): min/max must be visible to
// the networks' unqualified calls, so they are declared before the include.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 min(u16x2 a, u16x2 b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ u16x2 max(u16x2 a, u16x2 b) { return __builtin_elementwise_max(a, b); }

#include "robust_nets.h"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

using namespace p2p;

__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
  return max(min(a, b), min(max(a, b), c));
}
template <int CTRL>
__device__ __forceinline__ uint32_t dppm(uint32_t x) {
  return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(x), CTRL, 0xF, 0xF, true));
}

// MODE 0: sort64 only; 1: full L=4 median chain (sort64, flip, bmerge64, flip, max)
template <int MODE>
__global__ __launch_bounds__(256) void probe(uint32_t* out, int reps, uint32_t seed) {
  extern __shared__ uint32_t pad[];
  const int lane = threadIdx.x & 63, q = lane & 3;
  uint32_t v[64];
  uint32_t x = seed ^ (blockIdx.x * 1024 + threadIdx.x) * 0x9E3779B9u;
#pragma unroll
  for (int j = 0; j < 64; ++j) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; v[j] = x; }
  uint32_t acc = 0;
  for (int r = 0; r < reps; ++r) {
    net_sort64<true>(v);
    if constexpr (MODE == 1) {
      const uint32_t k1 = (q & 1) ? 0xFFFFFFFFu : 0u, k2 = (q & 2) ? 0xFFFFFFFFu : 0u;
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const uint32_t a = v[j], b = v[63 - j];
        v[j] = umed3(a, dppm<0xB1>(b), k1);
        v[63 - j] = umed3(b, dppm<0xB1>(a), k1);
      }
      net_bmerge64<true>(v);
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const uint32_t a = v[j], b = v[63 - j];
        v[j] = umed3(a, dppm<0x1B>(b), k2);
        v[63 - j] = umed3(b, dppm<0x1B>(a), k2);
      }
      uint32_t mx = v[0];
#pragma unroll
      for (int j = 1; j < 64; ++j) mx = max(mx, v[j]);
      acc += max(mx, dppm<0xB1>(mx));
    } else {
      acc += v[31];
    }
    // perturb so the next rep is not a sorted input
#pragma unroll
    for (int j = 0; j < 64; ++j) v[j] ^= (acc + j) * 0x2545F491u;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// MODE 2: the MODE 1 chain on packed 16-bit keys (hi16 pass of a two-pass
// radix median): a wave-tile covers 32 coordinates instead of 16.
__device__ __forceinline__ uint32_t u(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ u16x2 p16(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ u16x2 keep16(u16x2 a, u16x2 pa, bool hi) {
  const u16x2 lo = min(a, pa), h = max(a, pa);
  return hi ? h : lo;
}
template <int MODE>
__global__ __launch_bounds__(256) void probe16(uint32_t* out, int reps, uint32_t seed) {
  extern __shared__ uint32_t pad[];
  const int lane = threadIdx.x & 63, q = lane & 3;
  u16x2 v[64];
  uint32_t x = seed ^ (blockIdx.x * 1024 + threadIdx.x) * 0x9E3779B9u;
#pragma unroll
  for (int j = 0; j < 64; ++j) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; v[j] = p16(x); }
  uint32_t acc = 0;
  for (int r = 0; r < reps; ++r) {
    net_sort64<true>(v);
    const bool k1 = q & 1, k2 = q & 2;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const u16x2 a = v[j], b = v[63 - j];
      v[j] = keep16(a, p16(dppm<0xB1>(u(b))), k1);
      v[63 - j] = keep16(b, p16(dppm<0xB1>(u(a))), k1);
    }
    net_bmerge64<true>(v);
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const u16x2 a = v[j], b = v[63 - j];
      v[j] = keep16(a, p16(dppm<0x1B>(u(b))), k2);
      v[63 - j] = keep16(b, p16(dppm<0x1B>(u(a))), k2);
    }
    u16x2 mx = v[0];
#pragma unroll
    for (int j = 1; j < 64; ++j) mx = max(mx, v[j]);
    acc += u(max(mx, p16(dppm<0xB1>(u(mx)))));
#pragma unroll
    for (int j = 0; j < 64; ++j) v[j] = p16(u(v[j]) ^ ((acc + j) * 0x2545F491u));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int MODE>
static void run(int waves_per_cu, uint32_t* out, int reps) {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  // block = 4 waves (one per SIMD); blocks per CU pinned by LDS
  const int blocks_per_cu = waves_per_cu / 4;
  const size_t lds = 160 * 1024 / blocks_per_cu - 1024;
  auto kern = MODE == 2 ? probe16<MODE> : probe<MODE>;
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int grid = cus * blocks_per_cu;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, 0, out, 2, 1u);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, 0, out, reps, 7u);
  CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
  float ms = 0; CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double wave_tiles = (double)grid * 4 * reps;
  const double per_simd_tiles = wave_tiles / (cus * 4.0);
  printf("MODE %d waves/CU %2d: %.3f ms, %.1f ns per wave-tile per SIMD (%.0f cycles @2.4GHz)\n", MODE, waves_per_cu, ms,
         ms * 1e6 / per_simd_tiles, ms * 1e-3 / per_simd_tiles * 2.4e9);
}

int main() {
  uint32_t* out;
  CHECK(hipMalloc(&out, 256 * 1024 * 16 * sizeof(uint32_t)));
  for (int w : {4, 8, 12, 16}) run<0>(w, out, 2000);
  for (int w : {4, 8, 12, 16}) run<1>(w, out, 2000);
  for (int w : {4, 8, 12, 16}) run<2>(w, out, 2000);  // 32 coordinates per wave-tile
  return 0;
}
