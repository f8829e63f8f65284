// Lab (round 5): FedAvg with the peer streams staged by
// LDS-DMA through DEDICATED loader waves, against the product layout
// (fedavg.hip: one 4096-float tile per block, 16-B nontemporal VGPR loads).
//
// Why a split: one wave keeps at most 63 vector-memory instructions in
// flight (the 6-bit vmcnt), i.e. 63 KiB of LDS-DMA, and the guide's
// ldsdma-fill row puts one loader wave at ~25 GB/s per CU while 6.8 TB/s
// needs ~26.5 GB/s per CU.  Round 3's per-wave ring (tools/fedavg_dma.hip)
// made every wave both loader and consumer and ran at 6.03-6.34 TB/s.
//
// fedavg_split<L, C, S, TF, CONS>: a persistent block of L loader waves and
// C consumer waves per CU (or BPC blocks per CU) owns tiles b, b+G, b+2G...
// of TF floats.  A stage is one peer's slice of one tile (TF*4 bytes); the
// stages of a block run (tile, peer) in list order through a ring of S
// stages in LDS.  ONE barrier per stage: before barrier i the loaders wait
// (vmcnt) until stage i has landed, after it they refill the slot stage i-1
// used (the consumers finished reading it before the barrier) with stage
// i+S-1.  So S-2..S-1 stages are in flight per block at all times.  Consumer
// wave c owns floats [c*TF/C, (c+1)*TF/C) of the tile: ds_read_b128 of its
// part of stage i, then the adds in peer order from +0 (aggregation.py:15,
// 25-28), at the tile's last peer / K and the apply (:31-38) -- the
// product's per-coordinate op order, so the result is bit-identical.
// CONS=false: the consumers only pass the barriers (the loaders' ceiling for
// FedAvg's access pattern).
//
// Measurement tool, not product.  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//     -fhip-fp32-correctly-rounded-divide-sqrt -o tools/fedavg_split tools/fedavg_split.hip
// Run: tools/fedavg_split [K=256] [n=16777216 floats per peer] [reps=7]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));
#define GLOBAL __attribute__((address_space(1)))
#define CONSTANT __attribute__((address_space(4)))

__device__ __forceinline__ float apply_lr(float w, float lr, float m) { return __fadd_rn(w, __fmul_rn(lr, m)); }
__device__ __forceinline__ const float* peer_at(const float* const* t, int k) {
  return reinterpret_cast<const float*>(((const CONSTANT uint64_t*)t)[k]);
}

// ---- product layout (fedavg.hip full-tile path) ----
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
        x[u][v] = __builtin_nontemporal_load((const GLOBAL f4*)(peer_at(peers, k + u) + base + 1024 * v));
#pragma unroll
    for (int u = 0; u < UN; ++u)
#pragma unroll
      for (int v = 0; v < NV; ++v) acc[v] += x[u][v];
  }
  const float fk = (float)K;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    GLOBAL f4* wp = (GLOBAL f4*)(w + base + 1024 * v);
    f4 wv = *wp, r;
    r.x = apply_lr(wv.x, lr, acc[v].x / fk); r.y = apply_lr(wv.y, lr, acc[v].y / fk);
    r.z = apply_lr(wv.z, lr, acc[v].z / fk); r.w = apply_lr(wv.w, lr, acc[v].w / fk);
    *wp = r;
  }
}

// ---- loader / consumer split ----
// ds_read_b128 x RPW of this lane's part at LDS byte address a, waited.
template <int RPW>
__device__ __forceinline__ void lds_read_part(f4 (&x)[RPW], uint32_t a) {
  if constexpr (RPW == 1) {
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(x[0]) : "v"(a));
  } else if constexpr (RPW == 2) {
    asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:1024\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(x[0]), "=&v"(x[1]) : "v"(a));
  } else if constexpr (RPW == 4) {
    asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:1024\n\t"
                 "ds_read_b128 %2, %4 offset:2048\n\tds_read_b128 %3, %4 offset:3072\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3]) : "v"(a));
  } else {
    static_assert(RPW == 8, "RPW in {1,2,4,8}");
    asm volatile("ds_read_b128 %0, %8\n\tds_read_b128 %1, %8 offset:1024\n\t"
                 "ds_read_b128 %2, %8 offset:2048\n\tds_read_b128 %3, %8 offset:3072\n\t"
                 "ds_read_b128 %4, %8 offset:4096\n\tds_read_b128 %5, %8 offset:5120\n\t"
                 "ds_read_b128 %6, %8 offset:6144\n\tds_read_b128 %7, %8 offset:7168\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3]), "=&v"(x[4]), "=&v"(x[5]), "=&v"(x[6]),
                   "=&v"(x[7])
                 : "v"(a));
  }
}
template <int AUX>
__device__ __forceinline__ void dma16(const float* src, void* lds_dst) {
  __builtin_amdgcn_global_load_lds((GLOBAL void*)(const_cast<float*>(src)), (__attribute__((address_space(3))) void*)lds_dst,
                                   16, 0, AUX);
}

template <int L, int C, int S, int TF, bool CONS>
__global__ __launch_bounds__(64 * (L + C)) void fedavg_split(const float* const* __restrict__ peers, int K, long ntiles,
                                                             float* w, float lr) {
  static_assert(TF % (256 * L) == 0 && TF % (256 * C) == 0, "whole 1-KiB pieces per wave");
  static_assert(S >= 3, "ring of >= 3 stages");
  constexpr int PER = TF / 256 / L;  // DMA instructions per loader wave per stage
  constexpr int RPW = TF / 256 / C;  // ds_read_b128 per consumer lane per stage
  static_assert((S - 2) * PER <= 63, "vmcnt is 6 bits");
  // ring[S] stages, then the w image of the tile (each consumer DMAs its own part)
  __shared__ __attribute__((aligned(16))) float lds[(S + 1) * TF];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const long G = gridDim.x, b = blockIdx.x;
  if (b >= ntiles) return;  // block-uniform
  const long my_tiles = (ntiles - b + G - 1) / G;
  const long N = my_tiles * K;  // stages (= barriers) of this block

  if (wv < L) {
    // loader: stage j = (tile b + (j / K) * G, peer j % K) into slot j % S
    long ti = b; int ki = 0, si = 0; long issued = 0;
    auto issue = [&]() {
      const float* base = peer_at(peers, ki) + ti * (long)TF + (wv * PER) * 256 + lane * 4;
#pragma unroll
      for (int q = 0; q < PER; ++q) dma16<2 /* nt */>(base + q * 256, &lds[si * TF + (wv * PER + q) * 256]);
      ++issued;
      si = si + 1 == S ? 0 : si + 1;
      if (++ki == K) { ki = 0; ti += G; }
    };
    for (int d = 0; d < S - 1 && issued < N; ++d) issue();
    for (long i = 0; i < N; ++i) {
      if (i + S - 2 < N) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((S - 2) * PER) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // stage i landed; stage i-1's slot read
      if (issued < N) issue();       // into that slot
    }
    return;
  }
  const int cw = wv - L;
  const uint32_t base_lds = (uint32_t)(uintptr_t)&lds[0];
  const uint32_t my_off = (uint32_t)(cw * RPW * 256 + lane * 4) * 4u;
  const float fk = (float)K;
  int slot = 0;
  for (long t = b; t < ntiles; t += G) {
    float* wt = w + t * TF + cw * RPW * 256 + lane * 4;
    if (CONS) {
#pragma unroll
      for (int r = 0; r < RPW; ++r) dma16<0>(wt + r * 256, &lds[S * TF + (cw * RPW + r) * 256]);
    }
    f4 acc[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) acc[r] = f4{0.f, 0.f, 0.f, 0.f};  // +0 init (:15)
    for (int k = 0; k < K; ++k) {
      __builtin_amdgcn_s_barrier();
      if (CONS) {
        f4 x[RPW];
        lds_read_part<RPW>(x, base_lds + (uint32_t)slot * (TF * 4) + my_off);
#pragma unroll
        for (int r = 0; r < RPW; ++r) acc[r] += x[r];  // list order (:25-28)
      }
      slot = slot + 1 == S ? 0 : slot + 1;
    }
    if (CONS) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's w DMA (and last tile's stores)
      f4 wq[RPW];
      lds_read_part<RPW>(wq, base_lds + (uint32_t)(S * TF * 4) + my_off);
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        f4 o;
        o.x = apply_lr(wq[r].x, lr, acc[r].x / fk); o.y = apply_lr(wq[r].y, lr, acc[r].y / fk);
        o.z = apply_lr(wq[r].z, lr, acc[r].z / fk); o.w = apply_lr(wq[r].w, lr, acc[r].w / fk);
        *(GLOBAL f4*)(wt + r * 256) = o;  // (:31-38)
      }
    }
  }
}

// ---- same-box references: contiguous streams ----
template <int UN>
__global__ __launch_bounds__(256) void vgpr_roof(const f4* __restrict__ a, long n4, float* sink) {
  f4 s = {0, 0, 0, 0};
  const long stride = (long)gridDim.x * 256;
  long i = blockIdx.x * 256L + threadIdx.x;
  for (; i + (UN - 1) * stride < n4; i += UN * stride) {
    f4 x[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) x[u] = __builtin_nontemporal_load((const GLOBAL f4*)(a + i + u * stride));
#pragma unroll
    for (int u = 0; u < UN; ++u) s += x[u];
  }
  if (s.x == 1234.5f) sink[0] = s.y;
}
template <int D, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void dma_roof(const float* __restrict__ a, long pieces_per_wave, float* sink) {
  __shared__ __attribute__((aligned(16))) float ring[WAVES][D][256];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long gw = (long)blockIdx.x * WAVES + wv;
  const float* src = a + gw * pieces_per_wave * 256 + lane * 4;
  for (long p = 0; p < pieces_per_wave; ++p) {
    __builtin_amdgcn_global_load_lds((GLOBAL void*)(const_cast<float*>(src + p * 256)),
                                     (__attribute__((address_space(3))) void*)&ring[wv][p % D][0], 16, 0, 2);
    if (p >= D - 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D - 1) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (ring[wv][0][lane] == 1234.5f) sink[0] = 1.f;
}

__global__ void init(float* a, long n, uint32_t salt) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    a[i] = (float)(((i ^ salt) * 2654435761u) & 1023) * (1.0f / 1024) - 0.5f;
}

static int CUS;
struct Var {
  const char* name;
  int kind;  // 0 FedAvg (checked, bytes 4n(K+2)), 1 read-only FedAvg pattern (bytes 4nK), 2 contiguous read roof (4nK)
  void (*fn)(const float**, const float*, int, long, float*, float*);
};

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 256;
  const long n = argc > 2 ? atol(argv[2]) : 16L << 20;  // floats per peer; a multiple of 8192
  const int reps = argc > 3 ? atoi(argv[3]) : 7;
  if (n % 8192) { printf("n must be a multiple of 8192\n"); return 2; }
  float *slab, *w0, *w, *ref, *sink;
  CHECK(hipMalloc(&slab, 4L * K * n)); CHECK(hipMalloc(&w0, 4 * n)); CHECK(hipMalloc(&w, 4 * n));
  CHECK(hipMalloc(&ref, 4 * n)); CHECK(hipMalloc(&sink, 64));
  hipLaunchKernelGGL(init, dim3(8192), dim3(256), 0, 0, slab, (long)K * n, 7u);
  hipLaunchKernelGGL(init, dim3(8192), dim3(256), 0, 0, w0, n, 99u);
  std::vector<const float*> hp(K);
  for (int k = 0; k < K; ++k) hp[k] = slab + (long)k * n;
  const float** dp; CHECK(hipMalloc(&dp, sizeof(void*) * K));
  CHECK(hipMemcpy(dp, hp.data(), sizeof(void*) * K, hipMemcpyHostToDevice));
  CHECK(hipDeviceGetAttribute(&CUS, hipDeviceAttributeMultiprocessorCount, 0));
  CHECK(hipDeviceSynchronize());
#define VG(NAME, NV, UN) {NAME, 0, [](const float** p, const float*, int K, long n, float* w, float*) { \
    hipLaunchKernelGGL((fedavg_vgpr<NV, UN>), dim3(n / (1024 * NV)), dim3(256), 0, 0, p, K, n, w, 0.1f); }}
#define SP(NAME, L, C, S, TF, BPC, CONS) {NAME, CONS ? 0 : 1, [](const float** p, const float*, int K, long n, float* w, float*) { \
    hipLaunchKernelGGL((fedavg_split<L, C, S, TF, CONS>), dim3(CUS * BPC), dim3(64 * (L + C)), 0, 0, p, K, n / TF, w, 0.1f); }}
#define DR(NAME, D, W, BPC) {NAME, 2, [](const float**, const float* a, int K, long n, float*, float* s) { \
    const long waves = (long)CUS * BPC * W; const long ppw = (long)K * n / 256 / waves; \
    hipLaunchKernelGGL((dma_roof<D, W>), dim3(CUS * BPC), dim3(64 * W), 0, 0, a, ppw, s); }}
#define VR(NAME, UN, GRID) {NAME, 2, [](const float**, const float* a, int K, long n, float*, float* s) { \
    hipLaunchKernelGGL((vgpr_roof<UN>), dim3(GRID), dim3(256), 0, 0, (const f4*)a, (long)K * n / 4, s); }}
  std::vector<Var> vars = {
      VG("vgpr nv4 u8 (product)", 4, 8),
      SP("split L4 C8 S4 T8192", 4, 8, 4, 8192, 1, true),
      SP("split L2 C8 S4 T8192", 2, 8, 4, 8192, 1, true),
      SP("split L8 C8 S4 T8192", 8, 8, 4, 8192, 1, true),
      SP("split L4 C8 S3 T8192", 4, 8, 3, 8192, 1, true),
      SP("split L4 C8 S4 T8192 g2", 4, 8, 4, 8192, 2, true),
      SP("split L4 C8 S4 T8192 g4", 4, 8, 4, 8192, 4, true),
      SP("split L4 C8 S4 T8192 g8", 4, 8, 4, 8192, 8, true),
      SP("split L2 C4 S4 T8192", 2, 4, 4, 8192, 1, true),
      SP("split L4 C8 S8 T4096", 4, 8, 8, 4096, 1, true),
      SP("loadonly L4 S4 T8192", 4, 8, 4, 8192, 1, false),
      DR("dma roof D16 W8 x1 (contig)", 16, 8, 1),
      VR("vgpr roof u4 g8192 (contig)", 4, 8192),
  };
  // correctness: every FedAvg variant bit-identical to the product layout
  CHECK(hipMemcpy(ref, w0, 4 * n, hipMemcpyDeviceToDevice));
  vars[0].fn(dp, slab, K, n, ref, sink);
  std::vector<uint32_t> href(n), hw(n);
  CHECK(hipMemcpy(href.data(), ref, 4 * n, hipMemcpyDeviceToHost));
  bool all_ok = true;
  for (size_t v = 1; v < vars.size(); ++v) {
    if (vars[v].kind != 0) continue;
    CHECK(hipMemcpy(w, w0, 4 * n, hipMemcpyDeviceToDevice));
    vars[v].fn(dp, slab, K, n, w, sink);
    CHECK(hipGetLastError());
    CHECK(hipMemcpy(hw.data(), w, 4 * n, hipMemcpyDeviceToHost));
    long bad = 0;
    for (long i = 0; i < n; ++i) bad += hw[i] != href[i];
    printf("%-30s %s (%ld of %ld differ)\n", vars[v].name, bad ? "DIFF" : "bit-exact", bad, n);
    all_ok = all_ok && bad == 0;
    fflush(stdout);
  }
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  std::vector<std::vector<float>> ms(vars.size());
  for (int rep = 0; rep < reps; ++rep)  // interleaved: every variant once per rep
    for (size_t v = 0; v < vars.size(); ++v) {
      vars[v].fn(dp, slab, K, n, w, sink);
      CHECK(hipEventRecord(e0));
      vars[v].fn(dp, slab, K, n, w, sink);
      CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
      float t; CHECK(hipEventElapsedTime(&t, e0, e1));
      ms[v].push_back(t);
    }
  printf("K=%d n=%ld  FedAvg bytes 4n(K+2) = %.2f GB, read-only 4nK = %.2f GB, CUs %d\n", K, n,
         4.0 * n * (K + 2) / 1e9, 4.0 * n * K / 1e9, CUS);
  for (size_t v = 0; v < vars.size(); ++v) {
    std::sort(ms[v].begin(), ms[v].end());
    const double bytes = vars[v].kind == 0 ? 4.0 * n * (K + 2) : 4.0 * n * K;
    const float t = ms[v][ms[v].size() / 2];
    printf("%-30s median %8.3f ms  %7.1f GB/s  (%.1f%% of 8 TB/s)  best %.1f\n", vars[v].name, t,
           bytes / (t * 1e-3) / 1e9, bytes / (t * 1e-3) / 8e12 * 100, bytes / (ms[v][0] * 1e-3) / 1e9);
  }
  return all_ok ? 0 : 1;
}
