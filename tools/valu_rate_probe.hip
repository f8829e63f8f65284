// Probe: how many wave64 VALU instructions per cycle one SIMD retires, by the
// number of waves resident on it (the MI355X guide gives v_fma_f32 2 cycles
// on a SIMD-32 and 4 for one wave alone).  This decides whether the robust
// kernels' floor is "instructions x 4 cycles per SIMD" or "x 2 with >= 2
// waves ready" (DESIGN §3 K2).
//
// One block per CU (dynamic LDS pins it), 4*W waves per block = W waves per
// SIMD.  Each wave runs ITERS x 64 ops through inline asm: eight
// independent accumulators (IND) or one dependent chain (DEP).  Each wave
// reports its shader-clock cycles (clock64) around the loop.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_rate_probe tools/valu_rate_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int OP, bool DEP>
__global__ void probe(float* out, long long* cyc, long long* rt, int iters) {
  extern __shared__ float pad[];
  float a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = threadIdx.x * 1e-3f + j;
  const float x = threadIdx.x * 0.5f, y = blockIdx.x * 0.25f;
  const long long r0 = wall_clock64();
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 64; ++j) {
      float& r = DEP ? a[0] : a[j & 7];
      if constexpr (OP == 0) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(r) : "v"(x), "v"(y));
      else if constexpr (OP == 1) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(r) : "v"(x), "v"(y));
      else if constexpr (OP == 2) asm volatile("v_min_f32 %0, %0, %1" : "+v"(r) : "v"(x));
      else if constexpr (OP == 4) asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(r) : "v"(x), "v"(y));
      else if constexpr (OP == 5) asm volatile("v_med3_u32 %0, %0, %1, %2" : "+v"(r) : "v"(x), "v"(y));
      else if constexpr (OP == 6) asm volatile("v_min_u32 %0, %0, %1" : "+v"(r) : "v"(x));
      else asm volatile("v_add_f32 %0, %0, %1" : "+v"(r) : "v"(x));
    }
  }
  const long long t1 = clock64();
  const long long r1 = wall_clock64();
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += a[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) {
    cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
    rt[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = r1 - r0;
  }
}

template <int OP, bool DEP>
void run(const char* name, int cus, int w, int iters) {
  const int threads = 256 * w, waves = cus * 4 * w;
  float* out;
  long long *cyc, *rt;
  CHECK(hipMalloc(&rt, sizeof(long long) * waves));
  CHECK(hipMalloc(&out, sizeof(float) * cus * threads));
  CHECK(hipMalloc(&cyc, sizeof(long long) * waves));
  const size_t lds = 96 * 1024;  // one block per CU
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(probe<OP, DEP>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipLaunchKernelGGL((probe<OP, DEP>), dim3(cus), dim3(threads), lds, 0, out, cyc, rt, iters);  // warm
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL((probe<OP, DEP>), dim3(cus), dim3(threads), lds, 0, out, cyc, rt, iters);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  long long* h = (long long*)malloc(sizeof(long long) * waves);
  CHECK(hipMemcpy(h, cyc, sizeof(long long) * waves, hipMemcpyDeviceToHost));
  long long* hr = (long long*)malloc(sizeof(long long) * waves);
  CHECK(hipMemcpy(hr, rt, sizeof(long long) * waves, hipMemcpyDeviceToHost));
  int rate = 0;
  CHECK(hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0));  // kHz
  double avg = 0, avgr = 0;
  for (int i = 0; i < waves; ++i) { avg += h[i]; avgr += hr[i]; }
  avg /= waves;
  avgr /= waves;
  const double loop_ns = avgr / (rate * 1e3) * 1e9;  // one wave's loop in ns (constant-rate clock)
  const double per_wave = avg / (64.0 * iters);      // cycles between one wave's instructions
  const double per_simd = per_wave / w;              // cycles per instruction retired by the SIMD
  const double clk = avg / loop_ns;                  // shader GHz during the loop
  const double ns_simd = loop_ns / (64.0 * iters) / w;
  printf("%-8s %s waves/SIMD=%d  cyc/inst per wave=%.2f  per SIMD=%.2f  ns/inst per SIMD=%.3f  shader clock %.2f GHz"
         "  (loop %.3f ms, kernel %.3f ms)\n", name, DEP ? "dep" : "ind", w, per_wave, per_simd, ns_simd, clk,
         loop_ns * 1e-6, ms);
  free(hr);
  CHECK(hipFree(rt));
  free(h);
  CHECK(hipFree(out));
  CHECK(hipFree(cyc));
}

int main() {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int iters = 1 << 13;
  for (int w = 1; w <= 4; ++w) run<0, false>("max3", cus, w, iters);
  for (int w = 1; w <= 4; ++w) run<1, false>("med3", cus, w, iters);
  for (int w = 1; w <= 4; ++w) run<2, false>("min", cus, w, iters);
  for (int w = 1; w <= 4; ++w) run<3, false>("add", cus, w, iters);
  for (int w = 1; w <= 3; ++w) run<4, false>("max3u", cus, w, iters);
  for (int w = 1; w <= 3; ++w) run<5, false>("med3u", cus, w, iters);
  for (int w = 1; w <= 3; ++w) run<6, false>("minu", cus, w, iters);
  for (int w = 1; w <= 2; ++w) run<0, true>("max3", cus, w, iters);
  for (int w = 1; w <= 2; ++w) run<1, true>("med3", cus, w, iters);
  return 0;
}
