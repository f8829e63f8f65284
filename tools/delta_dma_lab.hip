// Lab (round 5): the trainer delta (delta = cur - prev; prev = cur, reference
// node/node.py:273-282) with cur / prev staged by LDS-DMA through dedicated
// loader waves -- the FedAvg split kernel's scheme with two streams per tile
// -- against the product layout (delta.hip: one float4 per lane, nt loads and
// stores).  Bit-checked (IEEE subtraction either way).  Measurement tool,
// not product.  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/delta_dma_lab tools/delta_dma_lab.hip
// Run: tools/delta_dma_lab [n floats = 268435456] [reps = 9]
// Round 6 (last session): every layout also with device-scope (sc1) buffer
// stores, the product's store policy since round 6 (delta.hip st4_tile), to
// ask again whether the DMA scheme loses once the stores stop costing extra.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));
#define GLOBAL __attribute__((address_space(1)))

__device__ __forceinline__ void st_nt(float* p, f4 v) { __builtin_nontemporal_store(v, (GLOBAL f4*)p); }
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
// ST < 0: nontemporal global store of v to base + off; else a buffer store
// with cache-policy bits ST (16 = sc1) over a wave-uniform base.
template <int ST>
__device__ __forceinline__ void st_pol(float* base, uint32_t off, f4 v) {
  if constexpr (ST < 0) {
    st_nt(base + off, v);
  } else {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7FFFFFF0, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), rs, off * 4u, 0, ST);
  }
}

template <int ST>
__global__ __launch_bounds__(256) void delta_vgpr(const float* cur, float* prev, float* delta, long n) {
  const long b0 = (long)blockIdx.x * 1024;
  const long i = b0 + threadIdx.x * 4;
  if (b0 + 1024 > n) return;
  const f4 c = __builtin_nontemporal_load((const GLOBAL f4*)(cur + i));
  const f4 p = __builtin_nontemporal_load((const GLOBAL f4*)(prev + i));
  st_pol<ST>(delta + b0, threadIdx.x * 4, c - p);
  st_pol<ST>(prev + b0, threadIdx.x * 4, c);
}

template <int AUX>
__device__ __forceinline__ void dma16(const float* src, void* lds_dst) {
  __builtin_amdgcn_global_load_lds((GLOBAL void*)(const_cast<float*>(src)), (__attribute__((address_space(3))) void*)lds_dst,
                                   16, 0, AUX);
}
template <int RPW>
__device__ __forceinline__ void lds_read_part(f4 (&x)[RPW], uint32_t a) {
  static_assert(RPW == 2 || RPW == 4, "RPW");
  if constexpr (RPW == 2) {
    asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:1024\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(x[0]), "=&v"(x[1]) : "v"(a));
  } else {
    asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:1024\n\t"
                 "ds_read_b128 %2, %4 offset:2048\n\tds_read_b128 %3, %4 offset:3072\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3]) : "v"(a));
  }
}

// stage 2t = cur of tile t, stage 2t+1 = prev of tile t (per block, tiles b, b+G, ...)
template <int L, int C, int S, int TF, int ST>
__global__ __launch_bounds__(64 * (L + C)) void delta_split(const float* cur, float* prev, float* delta, long ntiles) {
  constexpr int PER = TF / 256 / L, RPW = TF / 256 / C;
  static_assert((S - 2) * PER <= 63, "vmcnt");
  __shared__ __attribute__((aligned(16))) float lds[S * TF];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const long G = gridDim.x, b = blockIdx.x;
  if (b >= ntiles) return;
  const long N = (ntiles - b + G - 1) / G * 2;
  if (wv < L) {
    long ti = b; int si = 0, ki = 0; long issued = 0;
    auto issue = [&]() {
      const float* src = (ki == 0 ? cur : prev) + ti * (long)TF + (wv * PER) * 256 + lane * 4;
#pragma unroll
      for (int q = 0; q < PER; ++q) dma16<2>(src + q * 256, &lds[si * TF + (wv * PER + q) * 256]);
      ++issued;
      si = si + 1 == S ? 0 : si + 1;
      if (++ki == 2) { ki = 0; ti += G; }
    };
    for (int d = 0; d < S - 1 && issued < N; ++d) issue();
    for (long i = 0; i < N; ++i) {
      if (i + S - 2 < N) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((S - 2) * PER) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (issued < N) issue();
    }
    return;
  }
  const int cw = wv - L;
  const uint32_t lds0 = (uint32_t)(uintptr_t)&lds[0];
  const uint32_t mine = (uint32_t)(cw * RPW * 256 + lane * 4) * 4u;
  int slot = 0;
  for (long t = b; t < ntiles; t += G) {
    f4 c[RPW], p[RPW];
    __builtin_amdgcn_s_barrier();
    lds_read_part<RPW>(c, lds0 + (uint32_t)slot * (TF * 4) + mine);
    slot = slot + 1 == S ? 0 : slot + 1;
    __builtin_amdgcn_s_barrier();
    lds_read_part<RPW>(p, lds0 + (uint32_t)slot * (TF * 4) + mine);
    slot = slot + 1 == S ? 0 : slot + 1;
    const uint32_t o = (uint32_t)(cw * RPW * 256 + lane * 4);
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      st_pol<ST>(delta + t * (long)TF, o + r * 256, c[r] - p[r]);
      st_pol<ST>(prev + t * (long)TF, o + r * 256, c[r]);
    }
  }
}

__global__ void init(float* a, long n, unsigned s) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ s;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    a[i] = (float)(x & 0xFFFFFF) * 1e-6f - 8.0f;
  }
}

int CUS = 256;
struct Var { const char* name; void (*fn)(const float*, float*, float*, long); };

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 268435456L;
  const int reps = argc > 2 ? atoi(argv[2]) : 9;
  if (n % 8192) { printf("n must be a multiple of 8192\n"); return 2; }
  CHECK(hipDeviceGetAttribute(&CUS, hipDeviceAttributeMultiprocessorCount, 0));
  float *cur, *prev0, *prev, *delta, *ref_d, *ref_p;
  CHECK(hipMalloc(&cur, 4 * n)); CHECK(hipMalloc(&prev0, 4 * n)); CHECK(hipMalloc(&prev, 4 * n));
  CHECK(hipMalloc(&delta, 4 * n)); CHECK(hipMalloc(&ref_d, 4 * n)); CHECK(hipMalloc(&ref_p, 4 * n));
  hipLaunchKernelGGL(init, dim3(8192), dim3(256), 0, 0, cur, n, 1u);
  hipLaunchKernelGGL(init, dim3(8192), dim3(256), 0, 0, prev0, n, 2u);
#define SP(NAME, L, C, S, TF, BPC, ST) {NAME, [](const float* c, float* p, float* d, long n) { \
    hipLaunchKernelGGL((delta_split<L, C, S, TF, ST>), dim3(CUS * BPC), dim3(64 * (L + C)), 0, 0, c, p, d, n / TF); }}
#define VG(NAME, ST) {NAME, [](const float* c, float* p, float* d, long n) { \
    hipLaunchKernelGGL(delta_vgpr<ST>, dim3(n / 1024), dim3(256), 0, 0, c, p, d, n); }}
  std::vector<Var> vars = {
      VG("vgpr 1 float4/lane nt (r5)", -1),
      VG("vgpr 1 float4/lane sc1 (product)", 16),
      SP("split L4 C8 S4 T8192 nt", 4, 8, 4, 8192, 1, -1),
      SP("split L4 C8 S4 T8192 sc1", 4, 8, 4, 8192, 1, 16),
      SP("split L4 C8 S4 T8192 g2 sc1", 4, 8, 4, 8192, 2, 16),
      SP("split L4 C8 S6 T4096 sc1", 4, 8, 6, 4096, 1, 16),
      SP("split L4 C8 S6 T4096 g2 sc1", 4, 8, 6, 4096, 2, 16),
      SP("split L2 C4 S4 T4096 g4 sc1", 2, 4, 4, 4096, 4, 16),
      SP("split L4 C8 S4 T8192 sc1nt", 4, 8, 4, 8192, 1, 18),
  };
  // reference result (product layout), then every variant bit-compared
  CHECK(hipMemcpy(ref_p, prev0, 4 * n, hipMemcpyDeviceToDevice));
  vars[0].fn(cur, ref_p, ref_d, n);
  std::vector<uint32_t> hd(n), hp(n), rd(n), rp(n);
  CHECK(hipMemcpy(rd.data(), ref_d, 4 * n, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(rp.data(), ref_p, 4 * n, hipMemcpyDeviceToHost));
  for (size_t v = 1; v < vars.size(); ++v) {
    CHECK(hipMemcpy(prev, prev0, 4 * n, hipMemcpyDeviceToDevice));
    vars[v].fn(cur, prev, delta, n);
    CHECK(hipGetLastError());
    CHECK(hipMemcpy(hd.data(), delta, 4 * n, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(hp.data(), prev, 4 * n, hipMemcpyDeviceToHost));
    long bad = 0;
    for (long i = 0; i < n; ++i) bad += (hd[i] != rd[i]) + (hp[i] != rp[i]);
    printf("%-32s %s\n", vars[v].name, bad ? "DIFF" : "bit-exact");
    fflush(stdout);
  }
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  std::vector<std::vector<float>> ms(vars.size());
  for (int rep = 0; rep < reps; ++rep)
    for (size_t v = 0; v < vars.size(); ++v) {
      vars[v].fn(cur, prev, delta, n);
      CHECK(hipEventRecord(e0));
      vars[v].fn(cur, prev, delta, n);
      CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
      float t; CHECK(hipEventElapsedTime(&t, e0, e1));
      ms[v].push_back(t);
    }
  printf("n=%ld floats: 16 B per coordinate = %.2f GB per launch\n", n, 16.0 * n / 1e9);
  for (size_t v = 0; v < vars.size(); ++v) {
    std::sort(ms[v].begin(), ms[v].end());
    const float t = ms[v][ms[v].size() / 2];
    printf("%-32s median %7.3f ms  %7.1f GB/s  (%.1f%% of 8 TB/s)\n", vars[v].name, t, 16.0 * n / t / 1e6,
           16.0 * n / t / 1e6 / 80.0);
  }
  return 0;
}
