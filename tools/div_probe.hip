// Probe: is robust_nets.h div_const<D> (five instructions, or the IEEE
// division for |a| < 2^-118) the correctly rounded quotient a / D for EVERY
// float a?  The reference quotient is the
// double a / D rounded to float: rounding twice is innocuous for a division
// when the first precision is >= 2p + 2 (53 >= 50), subnormal results
// included (LLVM shrinks it to the f32 IEEE division, the sequence the
// kernels issued before).  NaN inputs compare as a class.  Also counts the
// unguarded four-instruction form (div_const_fast: what the guard is for)
// and the three-instruction form without v_div_fixup (what the fixup is for).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
//        -mno-amdgpu-ieee -fno-honor-nans -I p2pdl_amd/csrc -o tools/div_probe tools/div_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "robust_nets.h"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
using namespace p2p;

struct Miss {
  unsigned long long count, nofix, fast;
  uint32_t fast_max_abs;  // largest |a| (bits) the unguarded form misses
  uint32_t first[8], got[8], want[8];
};

__device__ __forceinline__ bool same(uint32_t a, uint32_t b) {
  const bool na = (a & 0x7FFFFFFFu) > 0x7F800000u, nb = (b & 0x7FFFFFFFu) > 0x7F800000u;
  return a == b || (na && nb);
}

template <int D>
__global__ void probe(uint64_t base, Miss* m) {
  const uint64_t i = base + static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint32_t bits = static_cast<uint32_t>(i);
  const float a = __uint_as_float(bits);
  const uint32_t want = __float_as_uint(static_cast<float>(static_cast<double>(a) / D));
  const uint32_t got = __float_as_uint(div_const<D>(a));
  constexpr float y = 1.0f / D;
  const float q0 = __fmul_rn(a, y);
  const uint32_t nofix = __float_as_uint(__builtin_fmaf(__builtin_fmaf(-q0, static_cast<float>(D), a), y, q0));
  if (!same(nofix, want)) atomicAdd(&m->nofix, 1ull);
  if (!same(__float_as_uint(div_const_fast<D>(a)), want)) {
    atomicAdd(&m->fast, 1ull);
    atomicMax(&m->fast_max_abs, bits & 0x7FFFFFFFu);
  }
  if (!same(got, want)) {
    const unsigned long long k = atomicAdd(&m->count, 1ull);
    if (k < 8) {
      m->first[k] = bits;
      m->got[k] = got;
      m->want[k] = want;
    }
  }
}

template <int D>
static void run() {
  Miss* m;
  CHECK(hipMalloc(&m, sizeof(Miss)));
  CHECK(hipMemset(m, 0, sizeof(Miss)));
  const uint64_t chunk = uint64_t(1) << 30;  // 2^22 blocks of 256 per launch
  for (uint64_t b = 0; b < (uint64_t(1) << 32); b += chunk)
    hipLaunchKernelGGL(probe<D>, dim3(chunk / 256), dim3(256), 0, 0, b, m);
  CHECK(hipGetLastError());
  Miss h;
  CHECK(hipMemcpy(&h, m, sizeof(Miss), hipMemcpyDeviceToHost));
  printf("{\"divisor\": %d, \"inputs\": 4294967296, \"mismatches\": %llu, \"unguarded_mismatches\": %llu, "
         "\"unguarded_max_abs_bits\": \"0x%08x\", \"unguarded_without_fixup\": %llu",
         D, h.count, h.fast, h.fast_max_abs, h.nofix);
  printf(", \"first\": [");
  for (unsigned k = 0; k < h.count && k < 8; ++k)
    printf("%s[\"0x%08x\", \"0x%08x\", \"0x%08x\"]", k ? ", " : "", h.first[k], h.got[k], h.want[k]);
  printf("]}\n");
  CHECK(hipFree(m));
}

int main() {
  run<154>();  // trimmed mean at K = 256, b = 51
  run<78>();   // K = 128, b = 25
  run<40>();   // K = 64, b = 12
  return 0;
}
