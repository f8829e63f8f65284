// Variant sweep for the K1 FedAvg kernel (measurement tool, not product).
// Builds standalone: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o fedavg_sweep fedavg_sweep.hip
// Times variants interleaved in ONE process (guide §5.4 rule 24) on a
// [K][n] slab far larger than the 256 MiB Infinity Cache, and two roofs:
// a pure streaming read and a float4 copy.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT> __device__ __forceinline__ f4 ld(const float* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const f4*>(p));
  else return *reinterpret_cast<const f4*>(p);
}

template <int VEC, int UNROLL, bool NT, bool STREAM_W>
__global__ __launch_bounds__(256) void fedavg_v(const float* const* __restrict__ peers, int K, long n,
                                                float* w, float lr) {
  constexpr int NV = VEC / 4;
  constexpr long TILE = 256L * VEC;
  const long ntiles = (n + TILE - 1) / TILE;
  const float fk = (float)K;
  for (long t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const long base = t * TILE + (long)threadIdx.x * VEC;
    if (base + VEC > n) continue;
    f4 acc[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) acc[v] = f4{0.f, 0.f, 0.f, 0.f};
    int k = 0;
    for (; k + UNROLL <= K; k += UNROLL) {
      f4 x[UNROLL][NV];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u)
#pragma unroll
        for (int v = 0; v < NV; ++v) x[u][v] = ld<NT>(peers[k + u] + base + 4 * v);
#pragma unroll
      for (int u = 0; u < UNROLL; ++u)
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[v] += x[u][v];
    }
    for (; k < K; ++k)
#pragma unroll
      for (int v = 0; v < NV; ++v) acc[v] += ld<NT>(peers[k] + base + 4 * v);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      f4 m = acc[v] / fk;
      f4 wv = *reinterpret_cast<f4*>(w + base + 4 * v);
      f4 r = wv + lr * m;
      if constexpr (STREAM_W) __builtin_nontemporal_store(r, reinterpret_cast<f4*>(w + base + 4 * v));
      else *reinterpret_cast<f4*>(w + base + 4 * v) = r;
    }
  }
}

// Block-interleaved: lane owns NV float4s at stride 256 float4 (every load
// instruction = one contiguous 1 KB per wave).  Optional per-block
// alignment check (what the product must do with a device pointer table).
template <int NV, int UNROLL, bool NT, bool CHECK>
__global__ __launch_bounds__(256) void fedavg_i(const float* const* __restrict__ peers, int K, long n,
                                                float* w, float lr) {
  constexpr long TILE = 1024L * NV;
  const long ntiles = (n + TILE - 1) / TILE;
  const float fk = (float)K;
  bool aligned = true;
  if constexpr (CHECK) {
    uintptr_t m = (uintptr_t)w;
    for (int k = 0; k < K; ++k) m |= (uintptr_t)peers[k];
    aligned = (m & 15) == 0;
  }
  for (long t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const long base = t * TILE + (long)threadIdx.x * 4;
    if (!aligned || t * TILE + TILE > n) continue;
    f4 acc[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) acc[v] = f4{0.f, 0.f, 0.f, 0.f};
    int k = 0;
    for (; k + UNROLL <= K; k += UNROLL) {
      f4 x[UNROLL][NV];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u)
#pragma unroll
        for (int v = 0; v < NV; ++v) x[u][v] = ld<NT>(peers[k + u] + base + 1024 * v);
#pragma unroll
      for (int u = 0; u < UNROLL; ++u)
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[v] += x[u][v];
    }
    for (; k < K; ++k)
#pragma unroll
      for (int v = 0; v < NV; ++v) acc[v] += ld<NT>(peers[k] + base + 1024 * v);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      f4 m = acc[v] / fk;
      f4 wv = *reinterpret_cast<f4*>(w + base + 1024 * v);
      *reinterpret_cast<f4*>(w + base + 1024 * v) = wv + lr * m;
    }
  }
}

// Peer-major "slab" variant: peers are rows of one [K][n] buffer (stride known)
template <int VEC, int UNROLL>
__global__ __launch_bounds__(256) void fedavg_slab(const float* __restrict__ slab, long stride, int K, long n,
                                                   float* w, float lr) {
  constexpr int NV = VEC / 4;
  constexpr long TILE = 256L * VEC;
  const long ntiles = (n + TILE - 1) / TILE;
  const float fk = (float)K;
  for (long t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const long base = t * TILE + (long)threadIdx.x * VEC;
    if (base + VEC > n) continue;
    f4 acc[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) acc[v] = f4{0.f, 0.f, 0.f, 0.f};
    const float* p = slab + base;
    for (int k = 0; k < K; k += UNROLL) {
      f4 x[UNROLL][NV];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u)
#pragma unroll
        for (int v = 0; v < NV; ++v) x[u][v] = ld<true>(p + (long)(k + u) * stride + 4 * v);
#pragma unroll
      for (int u = 0; u < UNROLL; ++u)
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[v] += x[u][v];
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      f4 m = acc[v] / fk;
      f4 wv = *reinterpret_cast<f4*>(w + base + 4 * v);
      *reinterpret_cast<f4*>(w + base + 4 * v) = wv + lr * m;
    }
  }
}

__global__ void read_roof(const f4* __restrict__ a, long n4, float* sink) {
  f4 s = {0, 0, 0, 0};
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256)
    s += __builtin_nontemporal_load(a + i);
  if (s.x == 1234.5f) sink[0] = s.y;  // never true: keeps the loads alive
}
__global__ void copy_roof(const f4* __restrict__ a, f4* b, long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) b[i] = a[i];
}
__global__ void init(float* a, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    a[i] = (float)((i * 2654435761u) & 1023) * (1.0f / 1024);
}

struct Var { const char* name; void (*fn)(hipStream_t); };

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 256;
  const long n = argc > 2 ? atol(argv[2]) : 32L * 1024 * 1024;
  const int rounds = argc > 3 ? atoi(argv[3]) : 3;
  // argv[4]: peer row pitch in floats (default n; -1 = one hipMalloc per peer);
  // argv[5]: 1 = only the product-like variants
  const long pitch = argc > 4 ? atol(argv[4]) : n;
  const bool few = argc > 5 && atoi(argv[5]) == 1;
  float* slab; float* w; float* tmp; float* sink;
  std::vector<const float*> hp(K);
  if (pitch > 0) {
    CHECK(hipMalloc(&slab, sizeof(float) * (size_t)K * pitch));
    hipLaunchKernelGGL(init, dim3(8192), dim3(256), 0, 0, slab, (long)K * pitch);
    for (int k = 0; k < K; ++k) hp[k] = slab + (long)k * pitch;
  } else {
    for (int k = 0; k < K; ++k) {
      float* r; CHECK(hipMalloc(&r, sizeof(float) * (size_t)n));
      hipLaunchKernelGGL(init, dim3(8192), dim3(256), 0, 0, r, n);
      hp[k] = r;
    }
    slab = const_cast<float*>(hp[0]);
  }
  CHECK(hipMalloc(&w, sizeof(float) * n));
  CHECK(hipMalloc(&tmp, sizeof(float) * n * 4));
  CHECK(hipMalloc(&sink, 64));
  hipLaunchKernelGGL(init, dim3(8192), dim3(256), 0, 0, w, n);
  const float** dp; CHECK(hipMalloc(&dp, sizeof(void*) * K));
  CHECK(hipMemcpy(dp, hp.data(), sizeof(void*) * K, hipMemcpyHostToDevice));
  CHECK(hipDeviceSynchronize());
  const double alg = 4.0 * n * (K + 2);

  static const float** P; static float* W; static long N; static int KK; static float* S; static float* T; static float* SL;
  P = dp; W = w; N = n; KK = K; S = sink; T = tmp; SL = slab;
#define V(NAME, VEC, UN, NT, SW, GRID) {NAME, [](hipStream_t s) { long tiles = (N + 256L*VEC - 1) / (256L*VEC); \
   int g = GRID ? GRID : (int)tiles; hipLaunchKernelGGL((fedavg_v<VEC, UN, NT, SW>), dim3(g), dim3(256), 0, s, P, KK, N, W, 0.1f); }}
#define VI(NAME, NV, UN, NT, CK, GRID) {NAME, [](hipStream_t s) { long tiles = (N + 1024L*NV - 1) / (1024L*NV); \
   int g = GRID ? GRID : (int)tiles; hipLaunchKernelGGL((fedavg_i<NV, UN, NT, CK>), dim3(g), dim3(256), 0, s, P, KK, N, W, 0.1f); }}
  std::vector<Var> vars = {
    V("v8u8nt g2048 (product r1)", 8, 8, true, false, 2048),
    V("v4u8nt onetile", 4, 8, true, false, 0),
    V("v4u8 plain onetile", 4, 8, false, false, 0),
    V("v4u16nt onetile", 4, 16, true, false, 0),
    V("v4u4nt onetile", 4, 4, true, false, 0),
    VI("i1u8nt onetile chk", 1, 8, true, true, 0),
    VI("i2u8nt onetile", 2, 8, true, false, 0),
    VI("i2u8nt onetile chk", 2, 8, true, true, 0),
    VI("i2u4nt onetile", 2, 4, true, false, 0),
    VI("i2u8 plain onetile", 2, 8, false, false, 0),
    VI("i4u4nt onetile", 4, 4, true, false, 0),
    VI("i4u4nt onetile chk", 4, 4, true, true, 0),
    VI("i4u8nt onetile", 4, 8, true, false, 0),
    VI("i2u8nt g4096 chk", 2, 8, true, true, 4096),
    VI("i2u8nt g8192 chk", 2, 8, true, true, 8192),
    VI("i4u4nt g4096 chk", 4, 4, true, true, 4096),
    VI("i1u16nt onetile chk", 1, 16, true, true, 0),
  };
  if (few) vars = {VI("i1u8nt onetile chk", 1, 8, true, true, 0), VI("i4u8nt onetile", 4, 8, true, false, 0)};
  printf("pitch %ld floats (%s)\n", pitch, pitch > 0 ? "one slab" : "one allocation per peer");

  std::vector<std::vector<float>> ms(vars.size());
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; ++r) {
    for (size_t v = 0; v < vars.size(); ++v) {
      vars[v].fn(0);  // warm
      CHECK(hipEventRecord(e0, 0));
      for (int i = 0; i < 3; ++i) vars[v].fn(0);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float t; CHECK(hipEventElapsedTime(&t, e0, e1));
      ms[v].push_back(t / 3);
    }
  }
  printf("K=%d n=%ld alg=%.2f GB per launch\n", K, n, alg / 1e9);
  for (size_t v = 0; v < vars.size(); ++v) {
    std::sort(ms[v].begin(), ms[v].end());
    printf("%-28s median %8.3f ms  %7.1f GB/s  (%.1f%% of 8 TB/s)  min %.3f\n", vars[v].name, ms[v][ms[v].size() / 2],
           alg / (ms[v][ms[v].size() / 2] * 1e-3) / 1e9, alg / (ms[v][ms[v].size() / 2] * 1e-3) / 8e12 * 100, ms[v][0]);
  }
  // roofs over the slab (K*n floats)
  const long n4 = (long)K * n / 4;
  for (int r = 0; r < (pitch > 0 && !few ? 2 : 0); ++r) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(read_roof, dim3(8192), dim3(256), 0, 0, (const f4*)slab, n4, sink);
    CHECK(hipEventRecord(e1, 0)); CHECK(hipEventSynchronize(e1));
    float t; CHECK(hipEventElapsedTime(&t, e0, e1));
    printf("read roof (nt, grid 8192): %.1f GB/s\n", K * n * 4.0 / (t * 1e-3) / 1e9);
    const long c4 = n;  // copy n*4 floats
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(copy_roof, dim3(8192), dim3(256), 0, 0, (const f4*)slab, (f4*)tmp, c4);
    CHECK(hipEventRecord(e1, 0)); CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&t, e0, e1));
    printf("copy roof (%ld MB each way): %.1f GB/s (read+write)\n", c4 * 16 / 1000000, 2.0 * c4 * 16 / (t * 1e-3) / 1e9);
  }
  return 0;
}
