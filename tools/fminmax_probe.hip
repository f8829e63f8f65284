// Probe: can the robust networks compare FLOATS instead of uint32 keys?
//  (1) semantics of v_min_f32 / v_max_f32 / v_med3_f32 / v_max3_f32 on the
//      cases where IEEE order and the total order could differ: -0 vs +0,
//      denormals (bits must pass through unchanged), +-inf;
//  (2) VALU throughput of the sort64 network on float vs uint32 operands.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-gpu-flush-denormals-to-zero -I p2pdl_amd/csrc \
//        -o tools/fminmax_probe tools/fminmax_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "robust_nets.h"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
using namespace p2p;

__global__ void semantics(const uint32_t* a, const uint32_t* b, uint32_t* out, int n) {
  const int i = threadIdx.x;
  if (i >= n) return;
  const float x = __uint_as_float(a[i]), y = __uint_as_float(b[i]);
  float r0, r1, r2, r3, r4, r5;
  const float ninf = -__builtin_inff(), pinf = __builtin_inff();
  asm volatile("v_min_f32 %0, %1, %2" : "=v"(r0) : "v"(x), "v"(y));
  asm volatile("v_max_f32 %0, %1, %2" : "=v"(r1) : "v"(x), "v"(y));
  asm volatile("v_med3_f32 %0, %1, %2, %3" : "=v"(r2) : "v"(x), "v"(y), "v"(ninf));
  asm volatile("v_med3_f32 %0, %1, %2, %3" : "=v"(r3) : "v"(x), "v"(y), "v"(pinf));
  asm volatile("v_max3_f32 %0, %1, %2, %3" : "=v"(r4) : "v"(x), "v"(y), "v"(ninf));
  asm volatile("v_min3_f32 %0, %1, %2, %3" : "=v"(r5) : "v"(x), "v"(y), "v"(pinf));
  out[6 * i + 0] = __float_as_uint(r0); out[6 * i + 1] = __float_as_uint(r1);
  out[6 * i + 2] = __float_as_uint(r2); out[6 * i + 3] = __float_as_uint(r3);
  out[6 * i + 4] = __float_as_uint(r4); out[6 * i + 5] = __float_as_uint(r5);
}

template <typename T>
__global__ __launch_bounds__(256) void sortbench(uint32_t* out, int reps, uint32_t seed) {
  T v[64];
  uint32_t x = seed ^ (blockIdx.x * 1024 + threadIdx.x) * 0x9E3779B9u;
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    if constexpr (sizeof(T) == 4 && T(0.5) != T(0)) v[j] = static_cast<T>(x >> 8);  // float: exact ints
    else v[j] = static_cast<T>(x);
  }
  T acc = 0;
  for (int r = 0; r < reps; ++r) {
    net_sort64<true>(v);
    acc = acc + v[31];
#pragma unroll
    for (int j = 0; j < 64; j += 2) { T t = v[j]; v[j] = v[63 - j]; v[63 - j] = t; }  // reverse pairs: unsorted again
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = static_cast<uint32_t>(acc);
}

template <typename T>
static float bench(const char* tag, uint32_t* out, int reps) {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = cus * 4;  // 16 waves per CU
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(sortbench<T>, dim3(grid), dim3(256), 0, 0, out, 2, 1u);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(sortbench<T>, dim3(grid), dim3(256), 0, 0, out, reps, 7u);
  CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
  float ms = 0; CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double per_simd = (double)grid * 4 * reps / (cus * 4.0);
  printf("sort64<%s>: %.3f ms, %.1f ns per wave-sort per SIMD\n", tag, ms, ms * 1e6 / per_simd);
  return ms;
}

int main() {
  const uint32_t cases[][2] = {
      {0x80000000u, 0x00000000u}, {0x00000000u, 0x80000000u},  // -0, +0
      {0x00000001u, 0x80000001u}, {0x80000001u, 0x00000001u},  // +-denormal
      {0x00000001u, 0x00000002u}, {0x007FFFFFu, 0x00800000u},  // denormal vs denormal / normal
      {0x80000000u, 0x80000001u}, {0x00000000u, 0x00000001u},  // zero vs tiny denormal
      {0x7F800000u, 0xFF800000u}, {0x3F800000u, 0x7F800000u},  // +-inf
      {0x80000000u, 0x80000000u}, {0x3F800000u, 0xBF800000u}};
  const int n = sizeof(cases) / sizeof(cases[0]);
  uint32_t ha[64], hb[64], hout[6 * 64];
  for (int i = 0; i < n; ++i) { ha[i] = cases[i][0]; hb[i] = cases[i][1]; }
  uint32_t *da, *db, *dout;
  CHECK(hipMalloc(&da, sizeof(ha))); CHECK(hipMalloc(&db, sizeof(hb))); CHECK(hipMalloc(&dout, sizeof(hout)));
  CHECK(hipMemcpy(da, ha, sizeof(ha), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(semantics, dim3(1), dim3(64), 0, 0, da, db, dout, n);
  CHECK(hipMemcpy(hout, dout, sizeof(hout), hipMemcpyDeviceToHost));
  // total-order keys: expected min / max bits
  auto key = [](uint32_t b) { return (b & 0x80000000u) ? ~b : (b | 0x80000000u); };
  int bad = 0;
  for (int i = 0; i < n; ++i) {
    const uint32_t lo = key(ha[i]) <= key(hb[i]) ? ha[i] : hb[i];
    const uint32_t hi = key(ha[i]) <= key(hb[i]) ? hb[i] : ha[i];
    const uint32_t* r = hout + 6 * i;
    const bool ok = r[0] == lo && r[1] == hi && r[2] == lo && r[3] == hi && r[4] == hi && r[5] == lo;
    bad += !ok;
    printf("%08x %08x -> min %08x max %08x med3(-inf) %08x med3(+inf) %08x max3 %08x min3 %08x  want lo %08x hi %08x %s\n",
           ha[i], hb[i], r[0], r[1], r[2], r[3], r[4], r[5], lo, hi, ok ? "ok" : "DIFF");
  }
  printf("semantics: %d of %d cases differ from the total order\n", bad, n);
  uint32_t* out;
  CHECK(hipMalloc(&out, 256 * 1024 * 4 * sizeof(uint32_t)));
  bench<uint32_t>("u32", out, 3000);
  bench<float>("f32", out, 3000);
  bench<uint32_t>("u32", out, 3000);
  bench<float>("f32", out, 3000);
  return 0;
}
