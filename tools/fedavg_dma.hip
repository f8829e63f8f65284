// Lab: FedAvg with the peer streams staged by LDS-DMA (global_load_lds_dwordx4
// nt: 1 KiB per wave instruction, no VGPR write-back) against the product
// layout (one tile per block, 16-B nontemporal loads into VGPRs).  The DMA
// read roof is 6.86-6.90 TB/s against 6.44-6.59 for VGPR loads
// (tools/dma_roof.hip, profiles/r03/dma).  Measurement tool, not product.
//
// DMA kernel: persistent; every wave works alone on wave-tiles of 256 x NV
// floats (lane l owns floats 4l..4l+3 of each 1-KiB piece -- exactly the 16 B
// its own DMA lane lands, so no cross-lane traffic) and walks the steps
// (tile, peer k, piece v) as one stream through a private ring of D pieces:
// D DMAs in flight, the oldest consumed (ds_read_b128) and its slot refilled
// with the step D ahead.  Per coordinate the peers are added in list order
// from +0, then / K and the apply -- the product's op order.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//        -fhip-fp32-correctly-rounded-divide-sqrt -o tools/fedavg_dma tools/fedavg_dma.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float apply_lr(float w, float lr, float m) { return __fadd_rn(w, __fmul_rn(lr, m)); }

// ---- product layout (fedavg.hip full-tile path, 4 float4 per lane, 8-deep) ----
template <int NV, int UN>
__global__ __launch_bounds__(256) void fedavg_vgpr(const float* const* __restrict__ peers, int K, long n, float* w,
                                                   float lr) {
  const long tile0 = (long)blockIdx.x * 1024 * NV;
  const long base = tile0 + threadIdx.x * 4;
  if (tile0 + 1024 * NV > n) return;
  f4 acc[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) acc[v] = f4{0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < K; k += UN) {
    f4 x[UN][NV];
#pragma unroll
    for (int u = 0; u < UN; ++u)
#pragma unroll
      for (int v = 0; v < NV; ++v)
        x[u][v] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(peers[k + u] + base + 1024 * v));
#pragma unroll
    for (int u = 0; u < UN; ++u)
#pragma unroll
      for (int v = 0; v < NV; ++v) acc[v] += x[u][v];
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    f4* wp = reinterpret_cast<f4*>(w + base + 1024 * v);
    f4 wv = *wp, r;
    r.x = apply_lr(wv.x, lr, acc[v].x / (float)K); r.y = apply_lr(wv.y, lr, acc[v].y / (float)K);
    r.z = apply_lr(wv.z, lr, acc[v].z / (float)K); r.w = apply_lr(wv.w, lr, acc[v].w / (float)K);
    *wp = r;
  }
}

// ---- LDS-DMA ----
template <int D>
__device__ __forceinline__ void dma_wait() {  // at most D-1 DMAs of this wave still outstanding
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D - 1) : "memory");
}
__device__ __forceinline__ f4 lds_read(uint32_t addr) {
  f4 x;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(x) : "v"(addr) : "memory");
  return x;
}

// w rows load through asm: the compiler would otherwise wait vmcnt(0) for
// them (it cannot count the loop's DMAs) and drain the ring every tile.
// Issued at the tile's start, they are complete long before the end (every
// step waits vmcnt(D-1), and loads return in order).
__device__ __forceinline__ f4 gload_async(const float* p) {
  f4 x;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(x) : "v"(p) : "memory");
  return x;
}

template <int D, int W, int NV>
__global__ __launch_bounds__(64 * W) void fedavg_dma(const float* const* __restrict__ peers, int K, long ntiles,
                                                     float* w, float lr) {
  __shared__ __attribute__((aligned(16))) float ring[W][D][256];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const long nw = (long)gridDim.x * W, gw = (long)blockIdx.x * W + wv;
  if (gw >= ntiles) return;
  const long my_tiles = (ntiles - gw + nw - 1) / nw;
  const long S = my_tiles * K * NV;  // steps of this wave
  const uint32_t lds0 = (uint32_t)(uintptr_t)&ring[wv][0][0] + lane * 16;
  // issue cursor
  long ti = gw; int ki = 0, vi = 0, si = 0; long issued = 0;
  auto issue = [&]() {
    const float* src = peers[ki] + ti * (256L * NV) + vi * 256 + lane * 4;
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(const_cast<float*>(src)),
                                     (__attribute__((address_space(3))) void*)&ring[wv][si][0], 16, 0, 2);
    ++issued;
    si = si + 1 == D ? 0 : si + 1;
    if (++vi == NV) { vi = 0; if (++ki == K) { ki = 0; ti += nw; } }
  };
  for (int d = 0; d < D && issued < S; ++d) issue();
  int su = 0;  // slot of the oldest outstanding step
  const float fk = (float)K;
  for (long t = gw; t < ntiles; t += nw) {
    f4 acc[NV], wq[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      acc[v] = f4{0.f, 0.f, 0.f, 0.f};
      wq[v] = gload_async(w + t * (256L * NV) + v * 256 + lane * 4);
    }
    for (int k = 0; k < K; ++k) {
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        if (issued < S) dma_wait<D>(); else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const f4 x = lds_read(lds0 + su * 1024);
        acc[v] += x;  // list order (aggregation.py:25-28)
        if (issued < S) issue();  // into the slot just read
        su = su + 1 == D ? 0 : su + 1;
      }
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      f4* wp = reinterpret_cast<f4*>(w + t * (256L * NV) + v * 256 + lane * 4);
      f4 r;
      r.x = apply_lr(wq[v].x, lr, acc[v].x / fk); r.y = apply_lr(wq[v].y, lr, acc[v].y / fk);
      r.z = apply_lr(wq[v].z, lr, acc[v].z / fk); r.w = apply_lr(wq[v].w, lr, acc[v].w / fk);
      *wp = r;
    }
  }
}

// Groups of G steps (NV = 1): one vmcnt wait, G ds_reads and the G peer
// pointers of the refill under ONE lgkmcnt wait, G adds, G DMAs.
template <int D, int W, int G>
__global__ __launch_bounds__(64 * W) void fedavg_dma2(const float* const* __restrict__ peers, int K, long ntiles,
                                                      float* w, float lr) {
  static_assert(D % G == 0, "whole groups per ring");
  __shared__ __attribute__((aligned(16))) float ring[W][D][256];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const long nw = (long)gridDim.x * W, gw = (long)blockIdx.x * W + wv;
  if (gw >= ntiles || K % G) return;
  const uint32_t lds0 = (uint32_t)(uintptr_t)&ring[wv][0][0] + lane * 16;
  // issue cursor: tile ti, peer ki, slot si (groups of G consecutive peers of one tile)
  long ti = gw; int ki = 0, si = 0;
  auto issue_group = [&](const float* const* pg) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float* src = pg[g] + ti * 256L + lane * 4;
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(const_cast<float*>(src)),
                                       (__attribute__((address_space(3))) void*)&ring[wv][si + g][0], 16, 0, 2);
    }
    si = si + G == D ? 0 : si + G;
    ki += G;
    if (ki == K) { ki = 0; ti += nw; }
  };
  for (int d = 0; d < D && ti < ntiles; d += G) {
    const float* pg[G];
#pragma unroll
    for (int g = 0; g < G; ++g) pg[g] = peers[ki + g];
    issue_group(pg);
  }
  int su = 0;
  const float fk = (float)K;
  for (long t = gw; t < ntiles; t += nw) {
    f4 acc = f4{0.f, 0.f, 0.f, 0.f};
    const f4 wq = gload_async(w + t * 256L + lane * 4);
    for (int k = 0; k < K; k += G) {
      const bool more = ti < ntiles;
      const float* pg[G];
      if (more) {
#pragma unroll
        for (int g = 0; g < G; ++g) pg[g] = peers[ki + g];
      }
      if (more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D - G) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      f4 x[G];
#pragma unroll
      for (int g = 0; g < G; ++g)
        asm volatile("ds_read_b128 %0, %1" : "=v"(x[g]) : "v"(lds0 + (su + g) * 1024) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int g = 0; g < G; ++g) acc += x[g];  // list order (aggregation.py:25-28)
      if (more) issue_group(pg);  // into the slots just read
      su = su + G == D ? 0 : su + G;
    }
    f4 r;
    r.x = apply_lr(wq.x, lr, acc.x / fk); r.y = apply_lr(wq.y, lr, acc.y / fk);
    r.z = apply_lr(wq.z, lr, acc.z / fk); r.w = apply_lr(wq.w, lr, acc.w / fk);
    *reinterpret_cast<f4*>(w + t * 256L + lane * 4) = r;
  }
}

__global__ void init(float* a, long n, uint32_t salt) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    a[i] = (float)(((i ^ salt) * 2654435761u) & 1023) * (1.0f / 1024) - 0.5f;
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 256;
  const long n = argc > 2 ? atol(argv[2]) : 16L << 20;  // per peer; must be a multiple of 4096
  float* slab; float* w0; float* w; float* ref;
  CHECK(hipMalloc(&slab, 4L * K * n)); CHECK(hipMalloc(&w0, 4 * n)); CHECK(hipMalloc(&w, 4 * n));
  CHECK(hipMalloc(&ref, 4 * n));
  hipLaunchKernelGGL(init, dim3(8192), dim3(256), 0, 0, slab, (long)K * n, 7u);
  hipLaunchKernelGGL(init, dim3(8192), dim3(256), 0, 0, w0, n, 99u);
  std::vector<const float*> hp(K);
  for (int k = 0; k < K; ++k) hp[k] = slab + (long)k * n;
  const float** dp; CHECK(hipMalloc(&dp, sizeof(void*) * K));
  CHECK(hipMemcpy(dp, hp.data(), sizeof(void*) * K, hipMemcpyHostToDevice));
  int cus = 0; CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CHECK(hipDeviceSynchronize());
  const double alg = 4.0 * n * (K + 2);
  struct Var { const char* name; void (*fn)(const float**, int, long, float*, int); };
  static int CUS; CUS = cus;
#define VG(NAME, NV, UN) {NAME, [](const float** p, int K, long n, float* w, int) { \
    hipLaunchKernelGGL((fedavg_vgpr<NV, UN>), dim3(n / (1024 * NV)), dim3(256), 0, 0, p, K, n, w, 0.1f); }}
#define DM(NAME, D, W, NV, BPC) {NAME, [](const float** p, int K, long n, float* w, int) { \
    hipLaunchKernelGGL((fedavg_dma<D, W, NV>), dim3(CUS * BPC), dim3(64 * W), 0, 0, p, K, n / (256 * NV), w, 0.1f); }}
#define D2(NAME, D, W, G, BPC) {NAME, [](const float** p, int K, long n, float* w, int) { \
    hipLaunchKernelGGL((fedavg_dma2<D, W, G>), dim3(CUS * BPC), dim3(64 * W), 0, 0, p, K, n / 256, w, 0.1f); }}
  std::vector<Var> vars = {
      VG("vgpr nv4 u8 (product)", 4, 8),
      D2("dma2 D8 W8 G4 x2", 8, 8, 4, 2), D2("dma2 D8 W16 G4 x1", 8, 16, 4, 1), D2("dma2 D4 W16 G4 x2", 4, 16, 4, 2),
      D2("dma2 D8 W16 G2 x1", 8, 16, 2, 1), D2("dma2 D16 W8 G8 x1", 16, 8, 8, 1), D2("dma2 D8 W4 G4 x4", 8, 4, 4, 4),
      D2("dma2 D4 W8 G4 x4", 4, 8, 4, 4), D2("dma2 D16 W4 G8 x2", 16, 4, 8, 2),
      DM("dma D8 W4 nv1 x2", 8, 4, 1, 2), DM("dma D16 W4 nv1 x2", 16, 4, 1, 2), DM("dma D8 W8 nv1 x2", 8, 8, 1, 2),
      DM("dma D16 W8 nv1 x1", 16, 8, 1, 1), DM("dma D8 W16 nv1 x1", 8, 16, 1, 1), DM("dma D8 W4 nv2 x2", 8, 4, 2, 2),
      DM("dma D16 W4 nv4 x2", 16, 4, 4, 2), DM("dma D4 W16 nv1 x2", 4, 16, 1, 2), DM("dma D8 W4 nv1 x4", 8, 4, 1, 4),
  };
  // correctness: every variant bit-identical to the product layout
  CHECK(hipMemcpy(ref, w0, 4 * n, hipMemcpyDeviceToDevice));
  vars[0].fn(dp, K, n, ref, 0);
  std::vector<uint32_t> href(n), hw(n);
  CHECK(hipMemcpy(href.data(), ref, 4 * n, hipMemcpyDeviceToHost));
  for (size_t v = 1; v < vars.size(); ++v) {
    CHECK(hipMemcpy(w, w0, 4 * n, hipMemcpyDeviceToDevice));
    vars[v].fn(dp, K, n, w, 0);
    CHECK(hipMemcpy(hw.data(), w, 4 * n, hipMemcpyDeviceToHost));
    long bad = 0;
    for (long i = 0; i < n; ++i) bad += hw[i] != href[i];
    printf("%-24s %s (%ld of %ld differ)\n", vars[v].name, bad ? "DIFF" : "bit-exact", bad, n);
  }
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  std::vector<std::vector<float>> ms(vars.size());
  for (int rep = 0; rep < 5; ++rep)
    for (size_t v = 0; v < vars.size(); ++v) {
      vars[v].fn(dp, K, n, w, 0);
      CHECK(hipEventRecord(e0));
      vars[v].fn(dp, K, n, w, 0);
      CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
      float t; CHECK(hipEventElapsedTime(&t, e0, e1));
      ms[v].push_back(t);
    }
  printf("K=%d n=%ld alg=%.2f GB per launch\n", K, n, alg / 1e9);
  for (size_t v = 0; v < vars.size(); ++v) {
    std::sort(ms[v].begin(), ms[v].end());
    const float t = ms[v][ms[v].size() / 2];
    printf("%-24s median %8.3f ms  %7.1f GB/s  (%.1f%% of 8 TB/s)  best %.1f\n", vars[v].name, t, alg / (t * 1e-3) / 1e9,
           alg / (t * 1e-3) / 8e12 * 100, alg / (ms[v][0] * 1e-3) / 1e9);
  }
  return 0;
}
