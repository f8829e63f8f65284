// Lab (round 6): the LDS-DMA split kernel's per-tile
// fixed cost.  The product (csrc/fedavg.hip fedavg_split_kernel) runs one
// 128-KiB-LDS block per 8192-float tile, one block resident per CU: every
// tile pays a block launch, the ring's prologue (the first stages' latency)
// and the epilogue (w DMA wait, / K, apply, stores) with nothing streaming
// on that CU in between.  profiles/r05/k_sweep: 0.758 / 0.781 / 0.854 of 8
// TB/s at K = 16 / 64 / 256, whatever the size.
//
// Variants, all bit-identical to the product layout (checked):
//   P   the product: L4 C8, 3-stage ring + w, T8192, grid = tiles
//   P4  the same with a 4-stage ring (160 KiB of LDS)
//   Q   persistent work queue: one block per CU claims tiles with a vector
//       atomic; the loaders stream tile j+1's stages during tile j's
//       epilogue (the ring runs across tile boundaries)
//   (Q with a 4-stage ring does not fit: 160 KiB + the tile queue)
//   H   half tiles: L2 C4, T4096, 3 stages + w = 64 KiB, so TWO blocks are
//       resident per CU and one streams while the other starts or ends
//   H4  H with 4 stages (80 KiB: two blocks fill the CU's 160 KiB)
//   HW  half tiles with the product's wave count: L4 C8, T4096 (2 reads
//       per consumer lane per stage), 64 KiB
//
// Measurement tool, not product.  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//     -o tools/split_fixed_lab tools/split_fixed_lab.hip
// Run: tools/split_fixed_lab K n reps   (n a multiple of 8192)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));
#define GLOBAL __attribute__((address_space(1)))
#define CONSTANT __attribute__((address_space(4)))
#define LDSAS __attribute__((address_space(3)))

__device__ __forceinline__ float apply_lr(float w, float lr, float m) { return __fadd_rn(w, __fmul_rn(lr, m)); }
__device__ __forceinline__ const float* peer_at(const float* const* t, int k) {
  return reinterpret_cast<const float*>(((const CONSTANT uint64_t*)t)[k]);
}
template <int AUX>
__device__ __forceinline__ void dma16(const float* src, void* lds_dst) {
  __builtin_amdgcn_global_load_lds((GLOBAL void*)(const_cast<float*>(src)), (LDSAS void*)lds_dst, 16, 0, AUX);
}
template <int RPW>
__device__ __forceinline__ void lds_read_part(f4 (&x)[RPW], uint32_t a) {
  if constexpr (RPW == 2) {
    asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:1024\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(x[0]), "=&v"(x[1]) : "v"(a));
  } else {
    static_assert(RPW == 4, "RPW in {2,4}");
    asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:1024\n\t"
                 "ds_read_b128 %2, %4 offset:2048\n\tds_read_b128 %3, %4 offset:3072\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3]) : "v"(a));
  }
}

template <int RPW>
__device__ __forceinline__ void epilogue(f4 (&acc)[RPW], float fk, float lr, uint32_t wlds, float* wt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's w DMA
  f4 wq[RPW];
  lds_read_part<RPW>(wq, wlds);
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    f4 o;
    o.x = apply_lr(wq[r].x, lr, acc[r].x / fk); o.y = apply_lr(wq[r].y, lr, acc[r].y / fk);
    o.z = apply_lr(wq[r].z, lr, acc[r].z / fk); o.w = apply_lr(wq[r].w, lr, acc[r].w / fk);
    *(GLOBAL f4*)(wt + r * 256) = o;  // (:31-38)
  }
}

// P / P4 / H / H4 / HW: one block per tile (grid = tiles), the product's loop.
template <int L, int C, int S, int TF>
__global__ __launch_bounds__(64 * (L + C)) void split_tile_blocks(const float* const* __restrict__ peers, int K,
                                                                  long ntiles, float* w, float lr) {
  constexpr int PER = TF / 256 / L, RPW = TF / 256 / C;
  static_assert((S - 2) * PER <= 63, "vmcnt");
  __shared__ __attribute__((aligned(16))) float lds[(S + 1) * TF];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const long t = blockIdx.x;
  const long N = K;
  if (wv < L) {
    int ki = 0, si = 0;
    long issued = 0;
    auto issue = [&]() {
      const float* src = peer_at(peers, ki) + t * (long)TF + (wv * PER) * 256 + lane * 4;
#pragma unroll
      for (int q = 0; q < PER; ++q) dma16<2>(src + q * 256, &lds[si * TF + (wv * PER + q) * 256]);
      ++issued; ++ki;
      si = si + 1 == S ? 0 : si + 1;
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
  float* wt = w + t * TF + cw * RPW * 256 + lane * 4;
#pragma unroll
  for (int r = 0; r < RPW; ++r) dma16<0>(wt + r * 256, &lds[S * TF + (cw * RPW + r) * 256]);
  f4 acc[RPW];
#pragma unroll
  for (int r = 0; r < RPW; ++r) acc[r] = f4{0.f, 0.f, 0.f, 0.f};
  int slot = 0;
  for (int k = 0; k < K; ++k) {
    __builtin_amdgcn_s_barrier();
    f4 x[RPW];
    lds_read_part<RPW>(x, lds0 + (uint32_t)slot * (TF * 4) + mine);
#pragma unroll
    for (int r = 0; r < RPW; ++r) acc[r] += x[r];
    slot = slot + 1 == S ? 0 : slot + 1;
  }
  epilogue<RPW>(acc, (float)K, lr, lds0 + (uint32_t)(S * TF * 4) + mine, wt);
}

// Q: persistent blocks, tiles claimed from a queue.  Tile 0 of block b
// is b; consumer wave 0 claims the block's next tile (a vector atomic on
// *counter, which the host sets to gridDim.x) when it starts a tile and
// writes it to tq[] after the tile's stage kW barrier; every loader wave
// reads it after barrier kR (> kW) of that tile, so it knows the next tile
// -- and whether there is one, i.e. its barrier count -- well before it
// issues that tile's first stage ((j+1)K - S + 1 > jK + kR for K >= 8).
// Every wave leaves once the queue is exhausted: the same number of
// barriers (K per tile) on both sides.
// The w path's parts: WD = w DMA (0 none, 1 plain, 2 nontemporal), ST = the
// epilogue's stores (0 none, 1 plain, 2 nontemporal).  WD 0 or ST 0 is a
// probe, not FedAvg (WD 0 applies to w = 0; ST 0 keeps the sums live by a
// store guarded by a NaN test that never holds).
// ST = 3: buffer stores with cache-policy bits AUX (bit 0 sc0, bit 1 nt,
// bit 4 sc1), through a descriptor at the tile's w base.
template <int L, int C, int S, int TF, int WD = 1, int ST = 1, int AUX = 0>
__global__ __launch_bounds__(64 * (L + C)) void split_queue(const float* const* __restrict__ peers, int K,
                                                            long ntiles, float* w, float lr, int* counter) {
  constexpr int PER = TF / 256 / L, RPW = TF / 256 / C;
  constexpr int kW = 2, kR = 4;
  static_assert((S - 2) * PER <= 63, "vmcnt");
  __shared__ __attribute__((aligned(16))) float lds[(S + 1) * TF];
  __shared__ long tq[4];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if ((long)blockIdx.x >= ntiles) return;  // host: grid <= ntiles
  if (wv < L) {
    long ti = blockIdx.x, tnext = -1;
    int ki = 0, si = 0;
    long issued = 0, N = K;
    auto issue = [&]() {
      if (ki == 0 && issued > 0) ti = tnext;
      const float* src = peer_at(peers, ki) + ti * (long)TF + (wv * PER) * 256 + lane * 4;
#pragma unroll
      for (int q = 0; q < PER; ++q) dma16<2>(src + q * 256, &lds[si * TF + (wv * PER + q) * 256]);
      ++issued;
      si = si + 1 == S ? 0 : si + 1;
      if (++ki == K) ki = 0;
    };
    for (int d = 0; d < S - 1 && issued < N; ++d) issue();
    for (long i = 0; i < N; ++i) {
      if (i + S - 2 < N) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((S - 2) * PER) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (i % K == kR) {  // the block's next tile (written after barrier jK + kW)
        tnext = __builtin_amdgcn_readfirstlane((int)tq[(i / K + 1) & 3]);
        if (tnext < ntiles) N += K;
      }
      if (issued < N) issue();
    }
    return;
  }
  const int cw = wv - L;
  const uint32_t lds0 = (uint32_t)(uintptr_t)&lds[0];
  const uint32_t mine = (uint32_t)(cw * RPW * 256 + lane * 4) * 4u;
  const float fk = (float)K;
  int slot = 0;
  long t = blockIdx.x;
  for (long j = 0;; ++j) {
    int claim = 0;
    if (cw == 0 && lane == 0) claim = atomicAdd(counter, 1);
    float* wt = w + t * TF + cw * RPW * 256 + lane * 4;
    if (WD) {
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        if (WD == 2) dma16<2>(wt + r * 256, &lds[S * TF + (cw * RPW + r) * 256]);
        else dma16<0>(wt + r * 256, &lds[S * TF + (cw * RPW + r) * 256]);
      }
    }
    f4 acc[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) acc[r] = f4{0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < K; ++k) {
      __builtin_amdgcn_s_barrier();
      if (k == kW && cw == 0) {
        if (lane == 0) tq[(j + 1) & 3] = claim;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      f4 x[RPW];
      lds_read_part<RPW>(x, lds0 + (uint32_t)slot * (TF * 4) + mine);
#pragma unroll
      for (int r = 0; r < RPW; ++r) acc[r] += x[r];
      slot = slot + 1 == S ? 0 : slot + 1;
    }
    if (ST == 0) {
      if (WD) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (acc[0].x != acc[0].x) *(GLOBAL f4*)wt = acc[0];  // never: the inputs hold no NaN
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's w DMA
      f4 wq[RPW];
      if (WD) {
        lds_read_part<RPW>(wq, lds0 + (uint32_t)(S * TF * 4) + mine);
      } else {
#pragma unroll
        for (int r = 0; r < RPW; ++r) wq[r] = f4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        f4 o;
        o.x = apply_lr(wq[r].x, lr, acc[r].x / fk); o.y = apply_lr(wq[r].y, lr, acc[r].y / fk);
        o.z = apply_lr(wq[r].z, lr, acc[r].z / fk); o.w = apply_lr(wq[r].w, lr, acc[r].w / fk);
        if (ST == 3) {
          const __amdgpu_buffer_rsrc_t rs =
              __builtin_amdgcn_make_buffer_rsrc(w + t * TF, 0, TF * 4, 0x00020000);
          __builtin_amdgcn_raw_buffer_store_b128(
              __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, o), rs,
              (cw * RPW * 256 + lane * 4 + r * 256) * 4, 0, AUX);
        } else if (ST == 2) {
          __builtin_nontemporal_store(o, (GLOBAL f4*)(wt + r * 256));
        } else {
          *(GLOBAL f4*)(wt + r * 256) = o;  // (:31-38)
        }
      }
    }
    t = __builtin_amdgcn_readfirstlane((int)tq[(j + 1) & 3]);
    if (t >= ntiles) break;
  }
}

__global__ void init(float* a, long n, uint32_t salt) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    a[i] = (float)(((i ^ salt) * 2654435761u) & 1023) * (1.0f / 1024) - 0.5f;
}

static int CUS;
static int* COUNTER;
struct Var {
  const char* name;
  void (*fn)(const float**, int, long, float*);
};

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 64;
  const long n = argc > 2 ? atol(argv[2]) : 11689984L;
  const int reps = argc > 3 ? atoi(argv[3]) : 9;
  if (n % 8192 || K < 8) { printf("n must be a multiple of 8192, K >= 8\n"); return 2; }
  float *slab, *w0, *w, *ref;
  CHECK(hipMalloc(&slab, 4L * K * n)); CHECK(hipMalloc(&w0, 4 * n)); CHECK(hipMalloc(&w, 4 * n));
  CHECK(hipMalloc(&ref, 4 * n)); CHECK(hipMalloc(&COUNTER, 64));
  hipLaunchKernelGGL(init, dim3(8192), dim3(256), 0, 0, slab, (long)K * n, 7u);
  hipLaunchKernelGGL(init, dim3(8192), dim3(256), 0, 0, w0, n, 99u);
  std::vector<const float*> hp(K);
  for (int k = 0; k < K; ++k) hp[k] = slab + (long)k * n;
  const float** dp; CHECK(hipMalloc(&dp, sizeof(void*) * K));
  CHECK(hipMemcpy(dp, hp.data(), sizeof(void*) * K, hipMemcpyHostToDevice));
  CHECK(hipDeviceGetAttribute(&CUS, hipDeviceAttributeMultiprocessorCount, 0));
  CHECK(hipDeviceSynchronize());
#define TB(NAME, L, C, S, TF) {NAME, [](const float** p, int K, long n, float* w) { \
    hipLaunchKernelGGL((split_tile_blocks<L, C, S, TF>), dim3(n / TF), dim3(64 * (L + C)), 0, 0, p, K, n / TF, w, 0.1f); }}
#define QU(NAME, L, C, S, TF) {NAME, [](const float** p, int K, long n, float* w) { \
    const long tiles = n / TF; const int g = (int)std::min<long>(tiles, CUS); \
    CHECK(hipMemcpyAsync(COUNTER, &g, 4, hipMemcpyHostToDevice, 0)); \
    hipLaunchKernelGGL((split_queue<L, C, S, TF>), dim3(g), dim3(64 * (L + C)), 0, 0, p, K, tiles, w, 0.1f, COUNTER); }}
#define QV(NAME, WD, ST) {NAME, [](const float** p, int K, long n, float* w) { \
    const long tiles = n / 8192; const int g = (int)std::min<long>(tiles, CUS); \
    CHECK(hipMemcpyAsync(COUNTER, &g, 4, hipMemcpyHostToDevice, 0)); \
    hipLaunchKernelGGL((split_queue<4, 8, 3, 8192, WD, ST>), dim3(g), dim3(64 * 12), 0, 0, p, K, tiles, w, 0.1f, COUNTER); }}
#define QB(NAME, AUX) {NAME, [](const float** p, int K, long n, float* w) { \
    const long tiles = n / 8192; const int g = (int)std::min<long>(tiles, CUS); \
    CHECK(hipMemcpyAsync(COUNTER, &g, 4, hipMemcpyHostToDevice, 0)); \
    hipLaunchKernelGGL((split_queue<4, 8, 3, 8192, 2, 3, AUX>), dim3(g), dim3(64 * 12), 0, 0, p, K, tiles, w, 0.1f, COUNTER); }}
  std::vector<Var> vars = {
      TB("P  L4C8 S3 T8192 (product)", 4, 8, 3, 8192),
      TB("P4 L4C8 S4 T8192", 4, 8, 4, 8192),
      QU("Q  queue L4C8 S3 T8192", 4, 8, 3, 8192),
      TB("H  L2C4 S3 T4096 (2/CU)", 2, 4, 3, 4096),
      TB("H4 L2C4 S4 T4096 (2/CU)", 2, 4, 4, 4096),
      TB("HW L4C8 S3 T4096 (2/CU)", 4, 8, 3, 4096),
      QV("QN queue, nt stores", 1, 2),
      QV("QNN queue, nt w DMA + nt stores", 2, 2),
      QV("QW queue, w DMA, no stores (probe)", 1, 0),
      QV("QS queue, stores, no w DMA (probe)", 0, 1),
      QV("QR queue, peers only (probe)", 0, 0),
      QB("QB0 nt w DMA, buffer store plain", 0),
      QB("QB2 nt w DMA, buffer store nt", 2),
      QB("QB3 nt w DMA, buffer store sc0 nt", 3),
      QB("QB16 nt w DMA, buffer store sc1", 16),
      QB("QB17 nt w DMA, buffer store sc0 sc1", 17),
      QB("QB18 nt w DMA, buffer store sc1 nt", 18),
      QB("QB19 nt w DMA, buffer store sc0 sc1 nt", 19),
  };
  // ONLY="P Q QR" (first token of each name) limits the variants
  if (const char* only = getenv("ONLY")) {
    std::vector<Var> keep;
    for (auto& v : vars) {
      std::string tok(v.name, strcspn(v.name, " "));
      if ((" " + std::string(only) + " ").find(" " + tok + " ") != std::string::npos) keep.push_back(v);
    }
    vars = keep;
  }
  CHECK(hipMemcpy(ref, w0, 4 * n, hipMemcpyDeviceToDevice));
  vars[0].fn(dp, K, n, ref);
  CHECK(hipGetLastError());
  std::vector<uint32_t> href(n), hw(n);
  CHECK(hipMemcpy(href.data(), ref, 4 * n, hipMemcpyDeviceToHost));
  bool all_ok = true;
  for (size_t v = 1; v < vars.size(); ++v) {
    if (strstr(vars[v].name, "(probe)")) continue;  // not FedAvg
    CHECK(hipMemcpy(w, w0, 4 * n, hipMemcpyDeviceToDevice));
    vars[v].fn(dp, K, n, w);
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
  for (int rep = 0; rep < reps; ++rep)
    for (size_t v = 0; v < vars.size(); ++v) {
      vars[v].fn(dp, K, n, w);
      CHECK(hipEventRecord(e0));
      vars[v].fn(dp, K, n, w);
      CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
      float t; CHECK(hipEventElapsedTime(&t, e0, e1));
      ms[v].push_back(t);
    }
  printf("K=%d n=%ld  FedAvg bytes 4n(K+2) = %.3f GB, CUs %d\n", K, n, 4.0 * n * (K + 2) / 1e9, CUS);
  for (size_t v = 0; v < vars.size(); ++v) {
    std::sort(ms[v].begin(), ms[v].end());
    const double bytes = 4.0 * n * (K + 2);  // every variant priced at FedAvg's bytes
    const float t = ms[v][ms[v].size() / 2];
    printf("%-30s median %8.4f ms  %.4f of 8 TB/s  best %.4f\n", vars[v].name, t, bytes / (t * 1e-3) / 8e12,
           bytes / (ms[v][0] * 1e-3) / 8e12);
  }
  fflush(stdout);
  return all_ok ? 0 : 1;
}
