// Lab (round 5): the K = 128 coordinate-wise median / trimmed mean (cfg4,
// SURVEY §8(d)) with the peer rows staged by LDS-DMA through DEDICATED loader
// waves -- the structure that took FedAvg past the VGPR-load rate
// (fedavg.hip fedavg_split_kernel) -- against the product kernel
// (robust.hip robust_flat_kernel: 128 VGPR loads of 256 B per wave).
//
// robust_stream_kernel<KP, RULE, NC>: one block per CU of NC loader + NC
// consumer waves.  Consumer p owns LDS slot p (KP peer rows x 64 floats) and
// the 64-coordinate tiles b*NC + p + j*G*NC; loader p fills slot p: it waits
// until consumer p has read the slot's previous tile (`empty[p]`), issues
// KP/4 global_load_lds_dwordx4 (each 1 KiB = 4 peer rows x 256 B, one row
// per 16 lanes), waits vmcnt(0) and publishes `full[p]`.  The consumer reads
// its KP keys (ds_read_b32, lane = coordinate), frees the slot, and runs the
// product's own networks on the floats (robust.hip special_floats; a wave
// holding a NaN re-runs on the keys, re-loading from HBM, as the product
// does) while its loader brings the next tile.  Flags are LDS words,
// generation counters; every spin is bounded and reports through `err`.
//
// Measurement tool, not product.  Built with the robust objects' flags:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//     -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero \
//     -mno-amdgpu-ieee -fno-honor-nans -mllvm -amdgpu-scalar-ir-passes=0 \
//     -Ip2pdl_amd/csrc -o tools/robust_stream tools/robust_stream.hip
// Run: tools/robust_stream [n=100000000] [reps=5]
#include "robust.hip"

// robust.hip's dispatcher names the K 129..256 family (robust_lds.hip), which
// this lab does not build or call.
extern "C" P2P_INTERNAL int64_t p2p_robust_lds_tile(int32_t, int32_t) { return 0; }
extern "C" P2P_INTERNAL void p2p_robust_lds_launch(const float* const*, const p2p_segment_t*, int32_t, int64_t,
                                                   int32_t, int32_t, int32_t, int64_t, float*, float*, float,
                                                   p2p_stream_t) {}

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

namespace p2p {

constexpr int64_t kSpinMax = int64_t(1) << 26;

__device__ __forceinline__ int lds_load_flag(int* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store_flag(int* f, int v) {
  __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// spin (bounded) until *f >= want; false on timeout
__device__ __forceinline__ bool wait_flag(int* f, int want) {
  for (int64_t i = 0; i < kSpinMax; ++i) {
    if (lds_load_flag(f) >= want) return true;
    __builtin_amdgcn_s_sleep(1);
  }
  return false;
}

template <int KP, int RULE, int NC>
__global__ __launch_bounds__(64 * 2 * NC, 1) void robust_stream_kernel(const float* const* __restrict__ peers,
                                                                       int64_t n, float* w, float* out, float lr,
                                                                       int* err) {
  constexpr int MODE = RULE == P2P_RULE_MEDIAN ? 1 : 2;
  constexpr int SLOT = KP * 64;  // floats per slot
  __shared__ __attribute__((aligned(16))) float slots[NC * SLOT];
  __shared__ int full[NC], empty[NC];
  const int wv = __builtin_amdgcn_readfirstlane(static_cast<int>(tid_x() >> 6));
  const int lane = tid_x() & 63;
  if (tid_x() < NC) {
    full[tid_x()] = 0;
    empty[tid_x()] = 0;
  }
  __syncthreads();
  const int64_t ntiles = n / 64;  // whole 64-coordinate tiles (the lab's n is a multiple of 64)
  const int64_t G = gridDim.x;
  if (wv < NC) {
    // ---- loader of slot p ----
    const int p = wv;
    const float* rowp[KP / 4];
#pragma unroll
    for (int q = 0; q < KP / 4; ++q) rowp[q] = table_at(peers, 4 * q + (lane >> 4)) + (lane & 15) * 4;
    int g = 0;
    for (int64_t t = bid_x() * NC + p; t < ntiles; t += G * NC, ++g) {
      if (!wait_flag(&empty[p], g)) { atomicOr(err, 1); return; }
      const int64_t c0 = t * 64;
#pragma unroll
      for (int q = 0; q < KP / 4; ++q)
        __builtin_amdgcn_global_load_lds((P2P_GLOBAL void*)(const_cast<float*>(rowp[q] + c0)),
                                         (__attribute__((address_space(3))) void*)&slots[p * SLOT + q * 256], 16, 0,
                                         2 /* nt */);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_store_flag(&full[p], g + 1);
    }
    return;
  }
  // ---- consumer of slot p ----
  const int p = wv - NC;
  int g = 0;
  for (int64_t t = bid_x() * NC + p; t < ntiles; t += G * NC, ++g) {
    if (!wait_flag(&full[p], g + 1)) { atomicOr(err, 2); return; }
    asm volatile("" ::: "memory");
    uint32_t v[KP];
#pragma unroll
    for (int j = 0; j < KP; ++j) v[j] = __float_as_uint(slots[p * SLOT + j * 64 + lane]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    lds_store_flag(&empty[p], g + 1);  // the loader may refill the slot now
    const int64_t c0 = t * 64;
    uint64_t nan = 0;
    float agg = special_floats<KP, RULE>(v, nan);
    if (__builtin_amdgcn_readfirstlane(static_cast<int>(nan != 0)))
      agg = robust_coord_keys<KP, RULE, MODE, false>(peers, KP, (KP * 2) / 10, c0, lane * 4u);
    const int64_t i = c0 + lane;
    if (out) stg(out + i, agg);
    if (w) stg(w + i, apply_lr(ldg(w + i), lr, agg));
  }
}

}  // namespace p2p

using namespace p2p;

__global__ void init(float* a, long n, uint32_t salt) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const uint32_t h = (uint32_t)((i ^ salt) * 2654435761u);
    a[i] = (float)(h & 0xFFFFF) * (1.0f / 1048576) - 0.5f;
  }
}

int main(int argc, char** argv) {
  constexpr int K = 128;
  const long n = argc > 1 ? atol(argv[1]) : 100000000L;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  if (n % 128) { printf("n must be a multiple of 128\n"); return 2; }
  float *slab, *w0, *w, *ref;
  int* err;
  CHECK(hipMalloc(&slab, 4L * K * n)); CHECK(hipMalloc(&w0, 4 * n)); CHECK(hipMalloc(&w, 4 * n));
  CHECK(hipMalloc(&ref, 4 * n)); CHECK(hipMalloc(&err, 4)); CHECK(hipMemset(err, 0, 4));
  hipLaunchKernelGGL(init, dim3(8192), dim3(256), 0, 0, slab, (long)K * n, 7u);
  hipLaunchKernelGGL(init, dim3(8192), dim3(256), 0, 0, w0, n, 99u);
  std::vector<const float*> hp(K);
  for (int k = 0; k < K; ++k) hp[k] = slab + (long)k * n;
  const float** dp; CHECK(hipMalloc(&dp, sizeof(void*) * K));
  CHECK(hipMemcpy(dp, hp.data(), sizeof(void*) * K, hipMemcpyHostToDevice));
  int cus = 0; CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CHECK(hipDeviceSynchronize());
  const double alg = 4.0 * n * (K + 2);
  struct Var { const char* name; int rule; int kind; int bpc; };
  // kind 0: product robust_flat_kernel (launch_one), 1: stream NC=4, 2: stream NC=2, 3: stream NC=6
  std::vector<Var> vars = {
      {"median product", P2P_RULE_MEDIAN, 0, 0}, {"median stream NC4", P2P_RULE_MEDIAN, 1, 1},
      {"median stream NC2 x2", P2P_RULE_MEDIAN, 2, 2},
      {"trimmed product", P2P_RULE_TRIMMED, 0, 0}, {"trimmed stream NC4", P2P_RULE_TRIMMED, 1, 1},
      {"trimmed stream NC2 x2", P2P_RULE_TRIMMED, 2, 2},
  };
  auto run = [&](const Var& v, float* wt) {
    if (v.kind == 0) {
      RobustArgs a{dp, nullptr, 0, 0, K, v.rule == P2P_RULE_TRIMMED ? (K * 2) / 10 : 0, n, wt, nullptr, 0.1f, 0};
      if (v.rule == P2P_RULE_MEDIAN) launch_one<K, P2P_RULE_MEDIAN, 1>(a);
      else launch_one<K, P2P_RULE_TRIMMED, 2>(a);
    } else if (v.kind == 1) {
      if (v.rule == P2P_RULE_MEDIAN)
        hipLaunchKernelGGL((robust_stream_kernel<K, P2P_RULE_MEDIAN, 4>), dim3(cus * v.bpc), dim3(512), 0, 0, dp, n,
                           wt, nullptr, 0.1f, err);
      else
        hipLaunchKernelGGL((robust_stream_kernel<K, P2P_RULE_TRIMMED, 4>), dim3(cus * v.bpc), dim3(512), 0, 0, dp, n,
                           wt, nullptr, 0.1f, err);
    } else {
      if (v.rule == P2P_RULE_MEDIAN)
        hipLaunchKernelGGL((robust_stream_kernel<K, P2P_RULE_MEDIAN, 2>), dim3(cus * v.bpc), dim3(256), 0, 0, dp, n,
                           wt, nullptr, 0.1f, err);
      else
        hipLaunchKernelGGL((robust_stream_kernel<K, P2P_RULE_TRIMMED, 2>), dim3(cus * v.bpc), dim3(256), 0, 0, dp, n,
                           wt, nullptr, 0.1f, err);
    }
  };
  bool all_ok = true;
  std::vector<uint32_t> href(n), hw(n);
  for (size_t i = 0; i < vars.size(); ++i) {
    if (vars[i].kind == 0) {
      CHECK(hipMemcpy(ref, w0, 4 * n, hipMemcpyDeviceToDevice));
      run(vars[i], ref);
      CHECK(hipMemcpy(href.data(), ref, 4 * n, hipMemcpyDeviceToHost));
      continue;
    }
    CHECK(hipMemcpy(w, w0, 4 * n, hipMemcpyDeviceToDevice));
    run(vars[i], w);
    CHECK(hipGetLastError());
    CHECK(hipMemcpy(hw.data(), w, 4 * n, hipMemcpyDeviceToHost));
    int e = 0;
    CHECK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
    long bad = 0;
    for (long j = 0; j < n; ++j) bad += hw[j] != href[j];
    printf("%-24s %s (%ld of %ld differ) err=%d\n", vars[i].name, bad || e ? "DIFF" : "bit-exact", bad, n, e);
    fflush(stdout);
    all_ok = all_ok && !bad && !e;
  }
  if (!all_ok) return 1;
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  std::vector<std::vector<float>> ms(vars.size());
  for (int rep = 0; rep < reps; ++rep)
    for (size_t i = 0; i < vars.size(); ++i) {
      run(vars[i], w);
      CHECK(hipEventRecord(e0));
      run(vars[i], w);
      CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
      float t; CHECK(hipEventElapsedTime(&t, e0, e1));
      ms[i].push_back(t);
    }
  printf("K=%d n=%ld alg=%.2f GB per launch (4n(K+2)), CUs %d\n", K, n, alg / 1e9, cus);
  for (size_t i = 0; i < vars.size(); ++i) {
    std::sort(ms[i].begin(), ms[i].end());
    const float t = ms[i][ms[i].size() / 2];
    printf("%-24s median %8.3f ms  %7.1f GB/s  (%.1f%% of 8 TB/s)  best %.3f ms\n", vars[i].name, t,
           alg / (t * 1e-3) / 1e9, alg / (t * 1e-3) / 8e12 * 100, ms[i][0]);
  }
  return 0;
}
