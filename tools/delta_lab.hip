// Lab: the trainer-delta kernel (csrc/delta.hip, 16 B per parameter: two
// streams in, two out) against a plain float4 copy (8 B per element) and
// layout variants, over 2^30 floats.  Measurement tool, not product.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/delta_lab tools/delta_lab.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));
#define G __attribute__((address_space(1)))

__device__ __forceinline__ f4 ld(const float* p) { return __builtin_nontemporal_load((const G f4*)p); }
__device__ __forceinline__ void st(float* p, f4 v) { __builtin_nontemporal_store(v, (G f4*)p); }
__device__ __forceinline__ void stp(float* p, f4 v) { *(G f4*)p = v; }

// V0: the product layout (tile per block, NV float4 per lane, stores interleaved).
// GROUP: all delta stores, then all prev stores.  PLAIN: prev stored without nt.
template <int NV, bool GROUP, bool PLAIN>
__global__ __launch_bounds__(256) void tile_k(const float* cur, float* prev, float* delta, long n) {
  const long base = (long)blockIdx.x * (1024 * NV) + 4 * threadIdx.x;
  f4 c[NV], p[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) c[v] = ld(cur + base + 1024 * v);
#pragma unroll
  for (int v = 0; v < NV; ++v) p[v] = ld(prev + base + 1024 * v);
  if (GROUP) {
#pragma unroll
    for (int v = 0; v < NV; ++v) st(delta + base + 1024 * v, c[v] - p[v]);
#pragma unroll
    for (int v = 0; v < NV; ++v) { if (PLAIN) stp(prev + base + 1024 * v, c[v]); else st(prev + base + 1024 * v, c[v]); }
  } else {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      st(delta + base + 1024 * v, c[v] - p[v]);
      if (PLAIN) stp(prev + base + 1024 * v, c[v]); else st(prev + base + 1024 * v, c[v]);
    }
  }
}

// Persistent grid-stride: each block walks tiles blockIdx, +grid, ...
template <int NV>
__global__ __launch_bounds__(256) void stride_k(const float* cur, float* prev, float* delta, long tiles) {
  for (long t = blockIdx.x; t < tiles; t += gridDim.x) {
    const long base = t * (1024 * NV) + 4 * threadIdx.x;
    f4 c[NV], p[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) c[v] = ld(cur + base + 1024 * v);
#pragma unroll
    for (int v = 0; v < NV; ++v) p[v] = ld(prev + base + 1024 * v);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      st(delta + base + 1024 * v, c[v] - p[v]);
      st(prev + base + 1024 * v, c[v]);
    }
  }
}

// Per-block contiguous chunk (each block owns CH tiles back to back).
template <int NV, int CH>
__global__ __launch_bounds__(256) void chunk_k(const float* cur, float* prev, float* delta, long tiles) {
  for (int k = 0; k < CH; ++k) {
    const long t = (long)blockIdx.x * CH + k;
    if (t >= tiles) return;
    const long base = t * (1024 * NV) + 4 * threadIdx.x;
    f4 c[NV], p[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) c[v] = ld(cur + base + 1024 * v);
#pragma unroll
    for (int v = 0; v < NV; ++v) p[v] = ld(prev + base + 1024 * v);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      st(delta + base + 1024 * v, c[v] - p[v]);
      st(prev + base + 1024 * v, c[v]);
    }
  }
}

// Round 5: the cache policy of loads and stores, for a
// copy and for the delta, same box, same sizes: LNT / SNT = nontemporal
// loads / stores, else plain (default policy).
template <bool LNT>
__device__ __forceinline__ f4 ldp(const float* p) {
  if constexpr (LNT) return __builtin_nontemporal_load((const G f4*)p);
  else return *(const G f4*)p;
}
template <bool SNT>
__device__ __forceinline__ void stpol(float* p, f4 v) {
  if constexpr (SNT) __builtin_nontemporal_store(v, (G f4*)p);
  else *(G f4*)p = v;
}
template <int NV, bool LNT, bool SNT>
__global__ __launch_bounds__(256) void copy_pol(const float* a, float* b, long n) {
  const long base = (long)blockIdx.x * (1024 * NV) + 4 * threadIdx.x;
  f4 c[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) c[v] = ldp<LNT>(a + base + 1024 * v);
#pragma unroll
  for (int v = 0; v < NV; ++v) stpol<SNT>(b + base + 1024 * v, c[v]);
}
// grid-stride float4 copy, one float4 per lane per trip (a STREAM-style copy)
template <bool LNT, bool SNT>
__global__ __launch_bounds__(256) void copy_gs(const float* a, float* b, long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256)
    stpol<SNT>(b + 4 * i, ldp<LNT>(a + 4 * i));
}
template <int NV, bool LNT, bool SNT, int BL>
__global__ __launch_bounds__(BL) void delta_pol(const float* cur, float* prev, float* delta, long n) {
  const long base = (long)blockIdx.x * (4 * BL * NV) + 4 * threadIdx.x;
  f4 c[NV], p[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) c[v] = ldp<LNT>(cur + base + 4 * BL * v);
#pragma unroll
  for (int v = 0; v < NV; ++v) p[v] = ldp<LNT>(prev + base + 4 * BL * v);
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    stpol<SNT>(delta + base + 4 * BL * v, c[v] - p[v]);
    stpol<SNT>(prev + base + 4 * BL * v, c[v]);
  }
}

// Roofs: copy (1 in, 1 out) and 2-in-2-out with 512-lane blocks.
template <int NV>
__global__ __launch_bounds__(256) void copy_k(const float* a, float* b, long n) {
  const long base = (long)blockIdx.x * (1024 * NV) + 4 * threadIdx.x;
  f4 c[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) c[v] = ld(a + base + 1024 * v);
#pragma unroll
  for (int v = 0; v < NV; ++v) st(b + base + 1024 * v, c[v]);
}

template <int NV>
__global__ __launch_bounds__(512) void tile512_k(const float* cur, float* prev, float* delta, long n) {
  const long base = (long)blockIdx.x * (2048 * NV) + 4 * threadIdx.x;
  f4 c[NV], p[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) c[v] = ld(cur + base + 2048 * v);
#pragma unroll
  for (int v = 0; v < NV; ++v) p[v] = ld(prev + base + 2048 * v);
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    st(delta + base + 2048 * v, c[v] - p[v]);
    st(prev + base + 2048 * v, c[v]);
  }
}

__global__ void init(float* a, long n, unsigned s) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    a[i] = (float)(((i + s) * 2654435761u) & 1023) * (1.0f / 1024);
}

static float* g_cur; static float* g_prev; static float* g_delta; static long g_n;

template <typename F>
static void timeit(const char* name, double bytes, F launch) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) launch();
  CHECK(hipDeviceSynchronize());
  const int reps = 20;
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) launch();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms; CHECK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  printf("%-28s %8.3f ms  %7.1f GB/s  %.4f\n", name, ms, bytes / ms * 1e-6, bytes / ms * 1e-6 / 8000.0);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 1L << 30;
  g_n = n;
  CHECK(hipMalloc(&g_cur, n * 4)); CHECK(hipMalloc(&g_prev, n * 4)); CHECK(hipMalloc(&g_delta, n * 4));
  init<<<4096, 256>>>(g_cur, n, 1); init<<<4096, 256>>>(g_prev, n, 7); init<<<4096, 256>>>(g_delta, n, 3);
  CHECK(hipDeviceSynchronize());
  int cus = 0; CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const double B16 = 16.0 * n, B8 = 8.0 * n;
  float *c = g_cur, *p = g_prev, *d = g_delta;
  // every kernel below needs n to be a multiple of its tile
  if (n % 16384) { printf("n must be a multiple of 16384\n"); return 1; }
  const bool policy = argc > 2 && atoi(argv[2]) == 1;
  if (policy) {  // round 5: load / store policy, copy vs delta, interleaved twice
    for (int rep = 0; rep < 2; ++rep) {
      timeit("hipMemcpyAsync D2D", B8, [&] { CHECK(hipMemcpyAsync(d, c, n * 4, hipMemcpyDeviceToDevice, 0)); });
      timeit("copy NV4 nt/nt", B8, [&] { copy_pol<4, true, true><<<n / 4096, 256>>>(c, d, n); });
      timeit("copy NV4 nt/plain", B8, [&] { copy_pol<4, true, false><<<n / 4096, 256>>>(c, d, n); });
      timeit("copy NV4 plain/nt", B8, [&] { copy_pol<4, false, true><<<n / 4096, 256>>>(c, d, n); });
      timeit("copy NV4 plain/plain", B8, [&] { copy_pol<4, false, false><<<n / 4096, 256>>>(c, d, n); });
      timeit("copy NV1 plain/plain", B8, [&] { copy_pol<1, false, false><<<n / 1024, 256>>>(c, d, n); });
      timeit("copy gs x8/CU plain/plain", B8, [&] { copy_gs<false, false><<<cus * 8, 256>>>(c, d, n / 4); });
      timeit("copy gs x32/CU plain/plain", B8, [&] { copy_gs<false, false><<<cus * 32, 256>>>(c, d, n / 4); });
      timeit("copy gs x32/CU nt/nt", B8, [&] { copy_gs<true, true><<<cus * 32, 256>>>(c, d, n / 4); });
      timeit("delta NV4 nt/nt (product)", B16, [&] { delta_pol<4, true, true, 256><<<n / 4096, 256>>>(c, p, d, n); });
      timeit("delta NV4 nt/plain", B16, [&] { delta_pol<4, true, false, 256><<<n / 4096, 256>>>(c, p, d, n); });
      timeit("delta NV4 plain/nt", B16, [&] { delta_pol<4, false, true, 256><<<n / 4096, 256>>>(c, p, d, n); });
      timeit("delta NV4 plain/plain", B16, [&] { delta_pol<4, false, false, 256><<<n / 4096, 256>>>(c, p, d, n); });
      timeit("delta512 NV2 nt/nt", B16, [&] { delta_pol<2, true, true, 512><<<n / 4096, 512>>>(c, p, d, n); });
      timeit("delta512 NV2 nt/plain", B16, [&] { delta_pol<2, true, false, 512><<<n / 4096, 512>>>(c, p, d, n); });
      timeit("delta NV1 nt/nt", B16, [&] { delta_pol<1, true, true, 256><<<n / 1024, 256>>>(c, p, d, n); });
      timeit("delta NV2 nt/nt", B16, [&] { delta_pol<2, true, true, 256><<<n / 2048, 256>>>(c, p, d, n); });
    }
    return 0;
  }
  for (int rep = 0; rep < 2; ++rep) {
    timeit("copy NV4", B8, [&] { copy_k<4><<<n / 4096, 256>>>(c, d, n); });
    timeit("copy NV8", B8, [&] { copy_k<8><<<n / 8192, 256>>>(c, d, n); });
    timeit("tile NV4 (product)", B16, [&] { tile_k<4, false, false><<<n / 4096, 256>>>(c, p, d, n); });
    timeit("tile NV4 group", B16, [&] { tile_k<4, true, false><<<n / 4096, 256>>>(c, p, d, n); });
    timeit("tile NV4 plain-prev", B16, [&] { tile_k<4, false, true><<<n / 4096, 256>>>(c, p, d, n); });
    timeit("tile NV2", B16, [&] { tile_k<2, false, false><<<n / 2048, 256>>>(c, p, d, n); });
    timeit("tile NV8", B16, [&] { tile_k<8, false, false><<<n / 8192, 256>>>(c, p, d, n); });
    timeit("tile512 NV2", B16, [&] { tile512_k<2><<<n / 4096, 512>>>(c, p, d, n); });
    timeit("tile512 NV4", B16, [&] { tile512_k<4><<<n / 8192, 512>>>(c, p, d, n); });
    for (int occ : {4, 8, 16, 32}) {
      char nm[64]; snprintf(nm, sizeof nm, "stride NV4 x%d/CU", occ);
      timeit(nm, B16, [&] { stride_k<4><<<cus * occ, 256>>>(c, p, d, n / 4096); });
    }
    timeit("chunk NV4 CH4", B16, [&] { chunk_k<4, 4><<<(n / 4096 + 3) / 4, 256>>>(c, p, d, n / 4096); });
    timeit("chunk NV4 CH16", B16, [&] { chunk_k<4, 16><<<(n / 4096 + 15) / 16, 256>>>(c, p, d, n / 4096); });
    timeit("chunk NV2 CH8", B16, [&] { chunk_k<2, 8><<<(n / 2048 + 7) / 8, 256>>>(c, p, d, n / 2048); });
  }
  return 0;
}
