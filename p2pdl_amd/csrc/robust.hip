// K2 -- coordinate-wise median / trimmed mean (+ optional apply) for gfx950.
//
// No reference implementation exists: the reference README.md:10 lists
// "Byzantine fault" as a TODO and aggregator/aggregation.py:7-46 only
// averages.  The rule is build-defined in SURVEY.md §8(a) row a8:
//   median : the key of rank (K-1)/2 under the IEEE total order on float bits
//   trimmed: b = floor(0.2 K); fp32 sum of sorted ranks b..K-b-1, ascending,
//            from +0, IEEE-divided by K-2b
// followed by the same apply as FedAvg (aggregation.py:36-38).
//
// Keys: float bits mapped to uint32 so the total order is unsigned order;
// a compare-exchange is one v_min_u32 + one v_max_u32 on VGPRs.  Networks are
// Batcher odd-even merge sorts / bitonic mergers generated (and 0-1-principle
// checked) by gen_networks.py into networks.inc.
//
// K <= 64: ONE LANE per coordinate (KP = next power of two, +inf pads; a
// network pruned to the wanted ranks when K == 64).  Loads: each wave
// instruction reads 256 contiguous bytes of one peer.
//
// K in 65..256: a WAVE GROUP per 64 coordinates -- P = 2 (K <= 128) or 4
// waves, wave q holding peers [64q, 64q+64).  Each wave sorts its 64 keys in
// registers (ascending or descending: bitonic block directions), then the
// group runs a bitonic merge: cross-wave half-cleaners through LDS (16
// registers per exchange round) and an in-register bmerge64.  ~75 VGPRs per
// lane -> 6 waves/SIMD, where one lane holding 128 keys needs ~150 VGPRs
// (3 waves/SIMD) and 256 keys do not fit.  The median of K = 64P stops after
// the first half-cleaner of the final merge: the lower P/2 waves then hold the
// K/2 smallest keys and the median is their maximum.  Trimmed sums run wave 0
// -> wave P-1 in ascending rank order, handing the partial sum on through LDS.
#include <stdlib.h>

#include "robust_nets.h"

namespace p2p {

constexpr int kRobustTile = 128;  // coordinates per block (one lane each, or 2 groups of 64)

template <int KP, int RULE, int MODE>
__device__ __forceinline__ float robust_coord(const float* const* __restrict__ peers, int K,
                                              int trim_b, int64_t i) {
  // Loads are unconditional (a pad slot re-reads peer 0, an L2 hit) so the
  // compiler can keep all of them in flight: a branch around each load made
  // it wait for every load before the branch merge (serialised, ~8x slower).
  uint32_t v[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    const bool real = (MODE != 0) || (j < K);  // MODE 1/2: K == KP
    const float* p = table_at(peers, real ? j : 0);
    v[j] = __float_as_uint(ldg_nt(p + i));
  }
  __builtin_amdgcn_sched_barrier(0);  // all KP loads in flight before the first use
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    const bool real = (MODE != 0) || (j < K);
    v[j] = real ? f2key(v[j]) : 0xFFFFFFFFu;  // pad: sorts after every real key
  }
  if constexpr (MODE == 0) {
    sort_full<KP>(v);
  } else {
    run_special<KP, MODE>(v);
  }
  if constexpr (RULE == P2P_RULE_MEDIAN) {
    if constexpr (MODE == 1) {
      return __uint_as_float(key2f(v[(KP - 1) / 2]));
    } else {
      const int r = (K - 1) / 2;
      uint32_t sel = v[0];
#pragma unroll
      for (int j = 1; j < KP; ++j) sel = (j == r) ? v[j] : sel;
      return __uint_as_float(key2f(sel));
    }
  } else {
    float acc = 0.f;  // ascending-rank sequential sum from +0
    if constexpr (MODE == 2) {
      constexpr int b = (KP * 2) / 10;  // floor(0.2 KP) for KP in {64,128,256}
#pragma unroll
      for (int j = b; j < KP - b; ++j) acc = __fadd_rn(acc, __uint_as_float(key2f(v[j])));
      return acc / static_cast<float>(KP - 2 * b);
    } else {
      const int hi = K - trim_b;
#pragma unroll
      for (int j = 0; j < KP; ++j) {
        const float x = __uint_as_float(key2f(v[j]));
        const float s = __fadd_rn(acc, x);
        acc = (j >= trim_b && j < hi) ? s : acc;
      }
      return acc / static_cast<float>(K - 2 * trim_b);
    }
  }
}

// ---- wave group, K in 65..256 ----------------------------------------------
// All-ascending bitonic merge across the P waves of a group: every wave sorts
// its 64 keys ascending; merge stage `size` (waves per merged block) starts
// with a FLIP (block position q against size-1-q, register j against the
// partner's register 63-j), then plain half-cleaners at wave distances
// size/4..1 (register j against j), then bmerge64 in registers.  No wave ever
// sorts descending, so no wave-dependent network and no phi copies of v[].
constexpr int kXchg = 16;  // registers exchanged through LDS per round

// LDS-only barrier: waits for this wave's LDS traffic, then s_barrier.  A
// __syncthreads() would also wait vmcnt(0) and drain the register prefetch of
// the next tile that is in flight during the sort.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ uint32_t keep(uint32_t a, uint32_t b, bool keep_min) {
  const uint32_t lo = min(a, b), hi = max(a, b);
  return keep_min ? lo : hi;  // keep_min is wave-uniform: one v_cndmask with an SGPR mask
}

// flip: v[j] = keep(v[j], partner.v[63-j]); rounds pair the low chunk
// [8c, 8c+8) with the mirrored high chunk [56-8c, 64-8c).
template <int H>
__device__ __forceinline__ void xchg_flip(uint32_t (&v)[H], uint32_t* lds, int wave, int partner,
                                          bool keep_min) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < H / 16; ++c) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      lds[(wave * kXchg + r) * 64 + lane] = v[8 * c + r];
      lds[(wave * kXchg + 8 + r) * 64 + lane] = v[H - 1 - 8 * c - r];
    }
    lds_barrier();
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      // partner's v[H-1-(8c+r)] sits in its high slot r; its v[8c+r] in low slot r
      v[8 * c + r] = keep(v[8 * c + r], lds[(partner * kXchg + 8 + r) * 64 + lane], keep_min);
      v[H - 1 - 8 * c - r] = keep(v[H - 1 - 8 * c - r], lds[(partner * kXchg + r) * 64 + lane], keep_min);
    }
    lds_barrier();
  }
}

// half-cleaner: v[j] = keep(v[j], partner.v[j])
template <int H>
__device__ __forceinline__ void xchg_half(uint32_t (&v)[H], uint32_t* lds, int wave, int partner,
                                          bool keep_min) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < H; c += kXchg) {
#pragma unroll
    for (int r = 0; r < kXchg; ++r) lds[(wave * kXchg + r) * 64 + lane] = v[c + r];
    lds_barrier();
#pragma unroll
    for (int r = 0; r < kXchg; ++r) v[c + r] = keep(v[c + r], lds[(partner * kXchg + r) * 64 + lane], keep_min);
    lds_barrier();
  }
}

constexpr int kGroupTile = 64;  // coordinates per wave-group tile

// Issue the 64 loads of one tile for this wave (raw float bits, no waits).
template <int H, int MODE>
__device__ __forceinline__ void group_issue(uint32_t (&nx)[H], const float* const* __restrict__ peers,
                                            int K, int wi, int64_t ic) {
#pragma unroll
  for (int j = 0; j < H; ++j) {  // unconditional loads (pads re-read peer 0)
    const int pj = wi * H + j;
    nx[j] = __float_as_uint(ldg_nt(table_at(peers, (MODE == 1 || pj < K) ? pj : 0) + ic));
  }
  // keep the 64 loads back to back: under register pressure the scheduler
  // otherwise pairs each load with its first use (64 serialised round trips)
  __builtin_amdgcn_sched_barrier(0);
}

template <int H> __device__ __forceinline__ void sort_h(uint32_t (&v)[H]);
template <> __device__ __forceinline__ void sort_h<64>(uint32_t (&v)[64]) { net_sort64<true>(v); }
template <> __device__ __forceinline__ void sort_h<128>(uint32_t (&v)[128]) { net_sort128<true>(v); }


// One 64-coordinate tile whose keys are in v[] (wave wi holds peers
// [H*wi, H*wi+H)).  MODE 1: median with K == H*P (stops after the final flip).
template <int H, int P, int RULE, int MODE>
__device__ __forceinline__ void group_tile(uint32_t (&v)[H], int K, int trim_b, int wi, int lane,
                                           int64_t i, bool live, float* w, float* out, float lr,
                                           uint32_t* lds) {
  sort_h<H>(v);
  bool done = false;
#pragma unroll
  for (int size = 2; size <= P; size *= 2) {
    const int q = wi % size, base = wi - q;
    xchg_flip<H>(v, lds, wi, base + size - 1 - q, q < size / 2);
    if constexpr (RULE == P2P_RULE_MEDIAN && MODE == 1) {
      if (size == P) {  // lower P/2 waves now hold the K/2 smallest keys
        uint32_t mx = v[0];
#pragma unroll
        for (int j = 1; j < H; ++j) mx = max(mx, v[j]);
        if constexpr (P == 4) {  // combine waves 0 and 1
          lds[wi * 64 + lane] = mx;
          lds_barrier();
          mx = max(mx, lds[(wi ^ 1) * 64 + lane]);
          lds_barrier();
        }
        if (wi == 0 && live) {
          const float agg = __uint_as_float(key2f(mx));
          if (out) stg(out + i, agg);
          if (w) stg(w + i, apply_lr(ldg(w + i), lr, agg));
        }
        done = true;
        break;
      }
    }
#pragma unroll
    for (int d = size / 4; d >= 1; d /= 2) xchg_half<H>(v, lds, wi, wi ^ d, (wi & d) == 0);
    bmerge<H>(v);
  }
  if (done) return;
  // fully sorted ascending across the group: wave wi holds ranks H*wi..H*wi+H-1
  if constexpr (RULE == P2P_RULE_MEDIAN) {
    const int r = (K - 1) / 2;
    if (wi == r / H) {
      const int rl = r % H;
      uint32_t sel = v[0];
#pragma unroll
      for (int j = 1; j < H; ++j) sel = (j == rl) ? v[j] : sel;
      if (live) {
        const float agg = __uint_as_float(key2f(sel));
        if (out) stg(out + i, agg);
        if (w) stg(w + i, apply_lr(ldg(w + i), lr, agg));
      }
    }
  } else {
    float* part = reinterpret_cast<float*>(lds);  // partial-sum hand-off
    const int hi = K - trim_b;
    float acc = 0.f;
#pragma unroll 1
    for (int qq = 0; qq < P; ++qq) {  // ascending rank order across the group
      if (wi == qq) {
        if (qq > 0) acc = part[lane];
#pragma unroll
        for (int j = 0; j < H; ++j) {
          const int g = qq * H + j;
          const float s = __fadd_rn(acc, __uint_as_float(key2f(v[j])));
          acc = (g >= trim_b && g < hi) ? s : acc;
        }
        part[lane] = acc;
      }
      lds_barrier();
    }
    if (wi == P - 1 && live) {
      const float agg = acc / static_cast<float>(K - 2 * trim_b);
      if (out) stg(out + i, agg);
      if (w) stg(w + i, apply_lr(ldg(w + i), lr, agg));
    }
  }
}

// Persistent wave group: block = P waves = one 64-coordinate tile at a time,
// grid-stride over tiles, next tile's loads prefetched into registers while
// the current tile is sorted and merged.
template <int H, int P, int RULE, int MODE, bool SEGS, bool PREFETCH>
__device__ __forceinline__ void robust_group_loop(const float* const* peers, const Seg* segs, int nseg,
                                                  int64_t ntiles, int K, int trim_b, int64_t n, float* w,
                                                  float* out, float lr, uint32_t* lds) {
  const int wi = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  auto locate = [&](int64_t t, const float* const*& pp, int64_t& nn, float*& ww, float*& oo, int64_t& lt) {
    if constexpr (SEGS) {
      const Seg s = load_segment(segs, nseg, t);
      pp = s.peers; nn = s.n; ww = s.w; oo = s.out; lt = t - s.tile_begin;
    } else {
      pp = peers; nn = n; ww = w; oo = out; lt = t;
    }
  };
  int64_t t = blockIdx.x;
  if (t >= ntiles) return;
  const float* const* pp; int64_t nn; float* ww; float* oo; int64_t lt;
  locate(t, pp, nn, ww, oo, lt);
  uint32_t nx[H];
  {
    const int64_t i = lt * kGroupTile + lane;
    group_issue<H, MODE>(nx, pp, K, wi, i < nn ? i : nn - 1);  // dead lanes re-read the last element
  }
  // PREFETCH: persistent grid-stride loop, next tile's loads in flight during
  // the sort.  Otherwise one tile per block (grid = tiles).
  const int64_t stride = PREFETCH ? static_cast<int64_t>(gridDim.x) : ntiles;
  for (; t < ntiles; t += stride) {
    const int64_t i = lt * kGroupTile + lane;
    const bool live = i < nn;
    float* cw = ww;
    float* co = oo;
    uint32_t v[H];
#pragma unroll
    for (int j = 0; j < H; ++j) {
      const uint32_t pad = (MODE == 1 || wi * H + j < K) ? 0u : 0xFFFFFFFFu;  // +inf pads sort last
      v[j] = f2key(nx[j]) | pad;
    }
    if constexpr (PREFETCH) {
      const int64_t tn = t + stride;
      if (tn < ntiles) {  // prefetch the next tile (uniform branch)
        locate(tn, pp, nn, ww, oo, lt);
        const int64_t i2 = lt * kGroupTile + lane;
        group_issue<H, MODE>(nx, pp, K, wi, i2 < nn ? i2 : nn - 1);
      }
    }
    group_tile<H, P, RULE, MODE>(v, K, trim_b, wi, lane, i, live, cw, co, lr, lds);
  }
}

// ---- kernels ---------------------------------------------------------------
// KP <= 128 (template arg): one lane per coordinate, 128-lane blocks.
// P in {2, 4} (GROUP kernels): 128*P-lane blocks.  A block covers kRobustTile
// coordinates either way.
template <int KP, int RULE, int MODE>
__device__ __forceinline__ void robust_one(const float* const* peers, int K, int trim_b, int64_t n,
                                           int64_t tile, float* w, float* out, float lr) {
  const int64_t i = tile * kRobustTile + threadIdx.x;
  if (i >= n) return;
  const float agg = robust_coord<KP, RULE, MODE>(peers, K, trim_b, i);
  if (out) stg(out + i, agg);
  if (w) stg(w + i, apply_lr(ldg(w + i), lr, agg));
}

template <int KP, int RULE, int MODE>
__global__ __launch_bounds__(kRobustTile) void robust_flat_kernel(
    const float* const* __restrict__ peers, int K, int trim_b, int64_t n, float* w, float* out,
    float lr) {
  robust_one<KP, RULE, MODE>(peers, K, trim_b, n, blockIdx.x, w, out, lr);
}

template <int KP, int RULE, int MODE>
__global__ __launch_bounds__(kRobustTile) void robust_segments_kernel(
    const Seg* __restrict__ segs, int nseg, int K, int trim_b, float lr) {
  const int64_t t = blockIdx.x;
  const Seg s = load_segment(segs, nseg, t);
  robust_one<KP, RULE, MODE>(s.peers, K, trim_b, s.n, t - s.tile_begin, s.w, s.out, lr);
}

template <int H, int P, int RULE, int MODE>
__global__ __launch_bounds__(64 * P) void robust_group_flat_kernel(
    const float* const* __restrict__ peers, int K, int trim_b, int64_t n, float* w, float* out,
    float lr) {
  __shared__ uint32_t lds[P * kXchg * 64];
  robust_group_loop<H, P, RULE, MODE, false, (P == 4)>(peers, nullptr, 0, ceil_div(n, kGroupTile), K,
                                                         trim_b, n, w, out, lr, lds);
}

template <int H, int P, int RULE, int MODE>
__global__ __launch_bounds__(64 * P) void robust_group_segments_kernel(
    const Seg* __restrict__ segs, int nseg, int64_t ntiles, int K, int trim_b, float lr) {
  __shared__ uint32_t lds[P * kXchg * 64];
  robust_group_loop<H, P, RULE, MODE, true, (P == 4)>(nullptr, segs, nseg, ntiles, K, trim_b, 0, nullptr,
                                                        nullptr, lr, lds);
}

struct RobustArgs {
  const float* const* peers;
  const Seg* segs;
  int nseg;
  int64_t tiles;
  int K, trim_b;
  int64_t n;
  float* w;
  float* out;
  float lr;
  hipStream_t stream;
};

template <int KP, int RULE, int MODE>
static void launch_one(const RobustArgs& a) {
  if (a.segs) {
    hipLaunchKernelGGL((robust_segments_kernel<KP, RULE, MODE>), dim3(static_cast<unsigned>(a.tiles)),
                       dim3(kRobustTile), 0, a.stream, a.segs, a.nseg, a.K, a.trim_b, a.lr);
  } else {
    hipLaunchKernelGGL((robust_flat_kernel<KP, RULE, MODE>),
                       dim3(static_cast<unsigned>(ceil_div(a.n, kRobustTile))), dim3(kRobustTile), 0,
                       a.stream, a.peers, a.K, a.trim_b, a.n, a.w, a.out, a.lr);
  }
}

template <int H, int P, int RULE, int MODE>
static void launch_group(const RobustArgs& a) {
  const int64_t ntiles = a.segs ? a.tiles : ceil_div(a.n, kGroupTile);
  // prefetching (P == 4) kernels are persistent: 2x the resident blocks
  // (12 waves/CU); the others launch one block per tile
  const int64_t cap = P == 4 ? 256 * (2 * 12 / P) : ntiles;
  const unsigned grid = static_cast<unsigned>(ntiles < cap ? ntiles : cap);
  if (a.segs) {
    hipLaunchKernelGGL((robust_group_segments_kernel<H, P, RULE, MODE>), dim3(grid), dim3(64 * P), 0,
                       a.stream, a.segs, a.nseg, a.tiles, a.K, a.trim_b, a.lr);
  } else {
    hipLaunchKernelGGL((robust_group_flat_kernel<H, P, RULE, MODE>), dim3(grid), dim3(64 * P), 0, a.stream,
                       a.peers, a.K, a.trim_b, a.n, a.w, a.out, a.lr);
  }
}

template <int KP, int RULE>
static void launch_kp(const RobustArgs& a) {
  if constexpr (KP == 64 || KP == 128) {
    if constexpr (RULE == P2P_RULE_MEDIAN) {
      if (a.K == KP) return launch_one<KP, RULE, 1>(a);
    } else {
      if (a.K == KP && a.trim_b == (KP * 2) / 10) return launch_one<KP, RULE, 2>(a);
    }
  }
  launch_one<KP, RULE, 0>(a);
}

template <int H, int P, int RULE>
static void launch_p(const RobustArgs& a) {
  if constexpr (RULE == P2P_RULE_MEDIAN) {
    if (a.K == H * P) return launch_group<H, P, RULE, 1>(a);
  }
  launch_group<H, P, RULE, 0>(a);
}

// Layout per (rule, K), from measurements on MI355X:
//   K <= 128     one lane per coordinate (median 68%, trimmed 56% of HBM peak
//                at K = 128; a 2-wave x 64-key group reached 61%)
//   K 129..256   4 waves x 64 keys with register prefetch of the next tile
//                (median 42%, trimmed 25% at K = 256; 2 waves x 128 keys
//                needs > 168 VGPRs and spills)
template <int RULE>
static void dispatch(const RobustArgs& a) {
  if (a.K <= 2) return launch_kp<2, RULE>(a);
  if (a.K <= 4) return launch_kp<4, RULE>(a);
  if (a.K <= 8) return launch_kp<8, RULE>(a);
  if (a.K <= 16) return launch_kp<16, RULE>(a);
  if (a.K <= 32) return launch_kp<32, RULE>(a);
  if (a.K <= 64) return launch_kp<64, RULE>(a);
  if (a.K <= 128) return launch_kp<128, RULE>(a);
  return launch_p<64, 4, RULE>(a);
}

}  // namespace p2p

using namespace p2p;

extern "C" P2P_INTERNAL int64_t p2p_robust_lds_tile(int32_t k, int32_t variant);
extern "C" P2P_INTERNAL void p2p_robust_lds_launch(const float* const* peers, const p2p_segment_t* segs,
                                                   int32_t nseg, int64_t tiles, int32_t k, int32_t rule,
                                                   int32_t trim_b, int64_t n, float* w, float* out, float lr,
                                                   int32_t variant, p2p_stream_t stream);

// Kernel family per K (tuning knob: p2p_set_robust_layout, or P2P_ROBUST_IMPL
// in the environment, read on first use).  Results are identical; the
// default is the fastest measured:
//   0 "auto"   K <= 128: one lane per coordinate (this file);
//              K 129..256: robust_lds.hip, 4 lanes x 64 keys
//   1 "lds"    robust_lds.hip for every K in 65..256 (4 lanes x 32 keys at K <= 128)
//   2 "lds2"   robust_lds.hip, 2 lanes x 64 keys at K <= 128
//   3 "group"  this file only: one lane (K <= 128) / 4-wave LDS group (K > 128)
//   4 "lds1"   robust_lds.hip, one lane x 128 keys (LDS-DMA staged) at K <= 128
//   5 "radix16" as auto, except median at K = 256: two-pass radix median with
//              packed 16-bit hi-half networks (robust_lds.hip, 128-coord tiles)
// (Measured and dropped: one LDS image per block with two blocks per CU for
// K > 128 -- 2 sorter waves per SIMD -- ran the same 26.6 ms as one block
// with two images: the K = 256 kernel is VALU-bound)
static int g_robust_impl = -1;
static int robust_impl() {
  if (g_robust_impl < 0) {
    const char* e = getenv("P2P_ROBUST_IMPL");
    int v = 0;
    if (e && e[0] == 'g') v = 3;
    else if (e && e[0] == 'l' && e[1] == 'd' && e[2] == 's') v = (e[3] == '2') ? 2 : (e[3] == '1') ? 4 : 1;
    else if (e && e[0] == 'r') v = 5;
    g_robust_impl = v;
  }
  return g_robust_impl;
}

// Which robust_lds.hip variant serves (rule, k, impl), or -1 for this file's kernels.
static int lds_variant(int rule, int k, int impl) {
  if (impl == 5 && k == 256 && rule == P2P_RULE_MEDIAN) return 3;
  if (k <= 64 || impl == 3) return -1;
  if (k > 128) return 0;
  return impl == 1 ? 0 : impl == 2 ? 1 : impl == 4 ? 2 : -1;
}

extern "C" int32_t p2p_set_robust_layout(int32_t layout) {
  if (layout < 0 || layout > 5) return P2P_ERR_INVALID;
  g_robust_impl = layout;
  return P2P_OK;
}

extern "C" P2P_INTERNAL int32_t p2p_robust_dispatch(const float* const* peers, const p2p_segment_t* segs,
                                       int32_t nseg, int64_t tiles, int32_t k, int32_t rule,
                                       int32_t trim_b, int64_t n, float* w, float* out, float lr,
                                       p2p_stream_t stream) {
  if (k < 1) return P2P_ERR_INVALID;
  if (k > 256) return P2P_ERR_UNSUPPORTED;
  if (rule == P2P_RULE_TRIMMED && (trim_b < 0 || k - 2 * trim_b <= 0)) return P2P_ERR_INVALID;
  if (rule != P2P_RULE_MEDIAN && rule != P2P_RULE_TRIMMED) return P2P_ERR_INVALID;
  const int var = lds_variant(rule, k, robust_impl());
  if (var >= 0) {
    p2p_robust_lds_launch(peers, segs, nseg, tiles, k, rule, trim_b, n, w, out, lr, var, stream);
  } else {
    RobustArgs a{peers, segs, nseg, tiles, k, trim_b, n, w, out, lr, static_cast<hipStream_t>(stream)};
    if (rule == P2P_RULE_MEDIAN) dispatch<P2P_RULE_MEDIAN>(a); else dispatch<P2P_RULE_TRIMMED>(a);
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? P2P_OK : static_cast<int32_t>(e);
}

extern "C" P2P_INTERNAL int64_t p2p_robust_tile_elems(int32_t rule, int32_t k) {
  const int var = lds_variant(rule, k, robust_impl());
  if (var >= 0) return p2p_robust_lds_tile(k, var);
  return k > 128 ? kGroupTile : kRobustTile;
}
