// Probe: do v_min3_f32 / v_max3_f32 / v_med3_f32 (as the fused networks
// emit them, robust_nets.h lo3 / hi3 / med3 on fk) select by the total order
// of the uint32 keys for EVERY operand order of every triple of special
// values (-0 / +0, denormals, +-inf, ties)?  The fused networks rely on it
// for bit-exact ranks (gen_networks.py); an equality test inside the
// hardware med3 that calls -0 == +0 would pick the wrong zero.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-gpu-flush-denormals-to-zero \
//        -mno-amdgpu-ieee -fno-honor-nans -I p2pdl_amd/csrc -o tools/med3_probe tools/med3_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "robust_nets.h"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
using namespace p2p;

static const uint32_t kVals[] = {0x80000000u, 0x00000000u, 0x00000001u, 0x80000001u, 0x007FFFFFu, 0x00800000u,
                                 0x3F800000u, 0xBF800000u, 0x7F800000u, 0xFF800000u, 0x3F800001u, 0xBF7FFFFFu};
constexpr int kN = sizeof(kVals) / sizeof(kVals[0]);

// one lane per ordered triple; out: min3, max3, med3 as the ascending (ASC)
// and descending networks issue them, plus med3 of the uint32 keys
__global__ void probe(const uint32_t* vals, uint32_t* out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= kN * kN * kN) return;
  const fk a{__uint_as_float(vals[t / (kN * kN)])}, b{__uint_as_float(vals[(t / kN) % kN])},
      c{__uint_as_float(vals[t % kN])};
  out[6 * t + 0] = __float_as_uint(lo3<true>(a, b, c).x);
  out[6 * t + 1] = __float_as_uint(hi3<true>(a, b, c).x);
  out[6 * t + 2] = __float_as_uint(med3(a, b, c).x);
  out[6 * t + 3] = __float_as_uint(lo3<false>(a, b, c).x);  // max3
  out[6 * t + 4] = __float_as_uint(hi3<false>(a, b, c).x);  // min3
  const fx d{a.x}, e{b.x}, f{c.x};
  out[6 * t + 5] = __float_as_uint(med3(d, e, f).x);
}

int main() {
  const int n = kN * kN * kN;
  uint32_t *dv, *dout;
  CHECK(hipMalloc(&dv, sizeof(kVals)));
  CHECK(hipMalloc(&dout, 6 * n * sizeof(uint32_t)));
  CHECK(hipMemcpy(dv, kVals, sizeof(kVals), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(probe, dim3((n + 255) / 256), dim3(256), 0, 0, dv, dout);
  CHECK(hipDeviceSynchronize());
  uint32_t* h = (uint32_t*)malloc(6 * n * sizeof(uint32_t));
  CHECK(hipMemcpy(h, dout, 6 * n * sizeof(uint32_t), hipMemcpyDeviceToHost));
  auto key = [](uint32_t x) { return (x & 0x80000000u) ? ~x : (x | 0x80000000u); };
  int bad = 0;
  for (int t = 0; t < n; ++t) {
    uint32_t v[3] = {kVals[t / (kN * kN)], kVals[(t / kN) % kN], kVals[t % kN]};
    for (int i = 0; i < 3; ++i)  // sort by key
      for (int j = i + 1; j < 3; ++j)
        if (key(v[j]) < key(v[i])) { uint32_t s = v[i]; v[i] = v[j]; v[j] = s; }
    const uint32_t* r = h + 6 * t;
    const bool ok = r[0] == v[0] && r[1] == v[2] && r[2] == v[1] && r[3] == v[2] && r[4] == v[0] && r[5] == v[1];
    if (!ok && bad++ < 20)
      printf("DIFF (%08x %08x %08x): min3 %08x max3 %08x med3 %08x | desc %08x %08x | fx med3 %08x; want %08x %08x %08x\n",
             kVals[t / (kN * kN)], kVals[(t / kN) % kN], kVals[t % kN], r[0], r[1], r[2], r[3], r[4], r[5], v[0],
             v[2], v[1]);
  }
  printf("med3_probe: %d ordered triples, %d mismatches\n", n, bad);
  return bad ? 1 : 0;
}
