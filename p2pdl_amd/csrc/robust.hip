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
// Design: one lane owns one coordinate.  Its K values are loaded (coalesced:
// 64 lanes read 256 contiguous bytes of one peer per instruction), mapped to
// uint32 total-order keys and sorted by a register-resident Batcher odd-even
// merge network (networks.inc, generated and 0-1-principle checked by
// gen_networks.py).  A compare-exchange is one v_min_u32 + one v_max_u32 on
// VGPRs -- no LDS round trips per stage.  When K equals the padded size KP
// and (for the trimmed mean) b = floor(0.2 K), a network pruned to the wanted
// ranks is used (median128: 2299 VALU ops vs 2942 for the full sort).
// Otherwise KP is the next power of two, slots K..KP-1 hold +inf pads
// (0xFFFFFFFF keys sort last) and the rank is picked with predicated selects.
//
// K in 129..256 runs on a LANE PAIR (256 live keys in one lane exceed the
// 512-entry register file and stall the register allocator): lane h of the
// pair holds peers [128h, 128h+128).  Lane 1 complements its keys so the same
// ascending sort128 network leaves it DESCENDING; one cross-lane half-cleaner
// (DPP quad_perm swap, min in lane 0 / max in lane 1) then puts the 128
// smallest keys in lane 0 and the 128 largest in lane 1, both bitonic, and a
// bmerge128 network sorts each lane.  The median of 256 is the max of lane 0
// after the half-cleaner (no merge needed).
#include "p2p_common.h"

#define P2P_CE(a, b)                     \
  do {                                   \
    const uint32_t lo_ = min((a), (b));  \
    (b) = max((a), (b));                 \
    (a) = lo_;                           \
  } while (0)
#define P2P_MIN(a, b) (a) = min((a), (b))
#define P2P_MAX(a, b) (b) = max((a), (b))

namespace p2p {
#include "networks.inc"

template <int KP> __device__ __forceinline__ void sort_full(uint32_t (&v)[KP]);
#define P2P_SORT(KP) \
  template <> __device__ __forceinline__ void sort_full<KP>(uint32_t (&v)[KP]) { net_sort##KP(v); }
P2P_SORT(2) P2P_SORT(4) P2P_SORT(8) P2P_SORT(16) P2P_SORT(32) P2P_SORT(64) P2P_SORT(128)
#undef P2P_SORT

// MODE 0: generic (full sort + runtime rank / trim);
// MODE 1: pruned median network for K == KP;
// MODE 2: pruned trimmed network for K == KP, b == floor(0.2 KP).
template <int KP, int MODE> __device__ __forceinline__ void run_special(uint32_t (&v)[KP]);
template <> __device__ __forceinline__ void run_special<64, 1>(uint32_t (&v)[64]) { net_median64(v); }
template <> __device__ __forceinline__ void run_special<128, 1>(uint32_t (&v)[128]) { net_median128(v); }
template <> __device__ __forceinline__ void run_special<64, 2>(uint32_t (&v)[64]) { net_trim64_b12(v); }
template <> __device__ __forceinline__ void run_special<128, 2>(uint32_t (&v)[128]) { net_trim128_b25(v); }

constexpr int kRobustTile = 128;  // coordinates per block (1 lane or a lane pair each)

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
    const uint32_t key = f2key(__float_as_uint(ldg_nt(p + i)));
    v[j] = real ? key : 0xFFFFFFFFu;  // pad: sorts after every real key
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

// ---- lane pair, K in 129..256 ---------------------------------------------
__device__ __forceinline__ uint32_t pair_swap(uint32_t x) {
  // DPP quad_perm [1,0,3,2]: exchange with the other lane of the pair
  return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(x), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float pair_swapf(float x) { return __uint_as_float(pair_swap(__float_as_uint(x))); }

// Returns the aggregate in the lane that owns it (*owner = true there).
template <int RULE>
__device__ __forceinline__ float robust_coord_pair(const float* const* __restrict__ peers, int K,
                                                   int trim_b, int64_t i, int h, bool* owner) {
  uint32_t v[128];
  const uint32_t m = h ? 0xFFFFFFFFu : 0u;
#pragma unroll
  for (int j = 0; j < 128; ++j) {
    const float* lo = table_at(peers, j);                   // K > 128: always valid
    const bool hi_real = (128 + j < K);
    const float* hi = table_at(peers, hi_real ? 128 + j : j);  // uniform, no branch
    const float* p = h ? hi : lo;
    const uint32_t key = f2key(__float_as_uint(ldg_nt(p + i)));
    v[j] = ((h == 0 || hi_real) ? key : 0xFFFFFFFFu) ^ m;  // lane 1: complemented
  }
  net_sort128(v);
#pragma unroll
  for (int j = 0; j < 128; ++j) {  // undo complement, then cross-lane half-cleaner
    const uint32_t x = v[j] ^ m;
    const uint32_t y = pair_swap(x);
    v[j] = h ? max(x, y) : min(x, y);
  }
  if constexpr (RULE == P2P_RULE_MEDIAN) {
    if (K == 256) {  // rank 127 = max of the lower half (lane 0)
      uint32_t mx = v[0];
#pragma unroll
      for (int j = 1; j < 128; ++j) mx = max(mx, v[j]);
      *owner = (h == 0);
      return __uint_as_float(key2f(mx));
    }
    net_bmerge128(v);
    const int r = (K - 1) / 2;  // global rank; lane h holds ranks 128h..128h+127
    const int rl = r - 128 * h;
    uint32_t sel = v[0];
#pragma unroll
    for (int j = 1; j < 128; ++j) sel = (j == rl) ? v[j] : sel;
    *owner = (rl >= 0 && rl < 128);
    return __uint_as_float(key2f(sel));
  } else {
    net_bmerge128(v);
    const int hi = K - trim_b;
    float acc = 0.f;  // pass 1: lane 0 sums its ranks
#pragma unroll
    for (int j = 0; j < 128; ++j) {
      const float s = __fadd_rn(acc, __uint_as_float(key2f(v[j])));
      acc = (h == 0 && j >= trim_b && j < hi) ? s : acc;
    }
    acc = pair_swapf(acc);  // lane 1 continues from lane 0's partial sum
#pragma unroll
    for (int j = 0; j < 128; ++j) {
      const int g = 128 + j;
      const float s = __fadd_rn(acc, __uint_as_float(key2f(v[j])));
      acc = (h == 1 && g >= trim_b && g < hi) ? s : acc;
    }
    *owner = (h == 1);
    return acc / static_cast<float>(K - 2 * trim_b);
  }
}

// ---- kernels ---------------------------------------------------------------
// KP <= 128: one lane per coordinate, 128-lane blocks.  KP == 256: lane pairs,
// 256-lane blocks.  Either way a block covers kRobustTile coordinates.
template <int KP, int RULE, int MODE>
__device__ __forceinline__ void robust_one(const float* const* peers, int K, int trim_b, int64_t n,
                                           int64_t tile, float* w, float* out, float lr) {
  if constexpr (KP <= 128) {
    const int64_t i = tile * kRobustTile + threadIdx.x;
    if (i >= n) return;
    const float agg = robust_coord<KP, RULE, MODE>(peers, K, trim_b, i);
    if (out) stg(out + i, agg);
    if (w) stg(w + i, apply_lr(ldg(w + i), lr, agg));
  } else {
    const int64_t i = tile * kRobustTile + (threadIdx.x >> 1);
    if (i >= n) return;  // both lanes of a pair leave together
    bool owner = false;
    const float agg = robust_coord_pair<RULE>(peers, K, trim_b, i, threadIdx.x & 1, &owner);
    if (owner) {
      if (out) stg(out + i, agg);
      if (w) stg(w + i, apply_lr(ldg(w + i), lr, agg));
    }
  }
}

template <int KP, int RULE, int MODE>
__global__ __launch_bounds__(KP <= 128 ? kRobustTile : 2 * kRobustTile) void robust_flat_kernel(
    const float* const* __restrict__ peers, int K, int trim_b, int64_t n, float* w, float* out,
    float lr) {
  robust_one<KP, RULE, MODE>(peers, K, trim_b, n, blockIdx.x, w, out, lr);
}

template <int KP, int RULE, int MODE>
__global__ __launch_bounds__(KP <= 128 ? kRobustTile : 2 * kRobustTile) void robust_segments_kernel(
    const Seg* __restrict__ segs, int nseg, int K, int trim_b, float lr) {
  const int64_t t = blockIdx.x;
  const Seg s = load_segment(segs, nseg, t);
  robust_one<KP, RULE, MODE>(s.peers, K, trim_b, s.n, t - s.tile_begin, s.w, s.out, lr);
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
  const dim3 block(KP <= 128 ? kRobustTile : 2 * kRobustTile);
  if (a.segs) {
    hipLaunchKernelGGL((robust_segments_kernel<KP, RULE, MODE>), dim3(static_cast<unsigned>(a.tiles)),
                       block, 0, a.stream, a.segs, a.nseg, a.K, a.trim_b, a.lr);
  } else {
    hipLaunchKernelGGL((robust_flat_kernel<KP, RULE, MODE>),
                       dim3(static_cast<unsigned>(ceil_div(a.n, kRobustTile))), block, 0, a.stream,
                       a.peers, a.K, a.trim_b, a.n, a.w, a.out, a.lr);
  }
}

template <int KP, int RULE>
static void launch_kp(const RobustArgs& a) {
  if constexpr (KP >= 64 && KP <= 128) {
    if constexpr (RULE == P2P_RULE_MEDIAN) {
      if (a.K == KP) return launch_one<KP, RULE, 1>(a);
    } else {
      if (a.K == KP && a.trim_b == (KP * 2) / 10) return launch_one<KP, RULE, 2>(a);
    }
  }
  launch_one<KP, RULE, 0>(a);
}

template <int RULE>
static void dispatch(const RobustArgs& a) {
  if (a.K <= 2) return launch_kp<2, RULE>(a);
  if (a.K <= 4) return launch_kp<4, RULE>(a);
  if (a.K <= 8) return launch_kp<8, RULE>(a);
  if (a.K <= 16) return launch_kp<16, RULE>(a);
  if (a.K <= 32) return launch_kp<32, RULE>(a);
  if (a.K <= 64) return launch_kp<64, RULE>(a);
  if (a.K <= 128) return launch_kp<128, RULE>(a);
  return launch_kp<256, RULE>(a);
}

}  // namespace p2p

using namespace p2p;

extern "C" P2P_INTERNAL int32_t p2p_robust_dispatch(const float* const* peers, const p2p_segment_t* segs,
                                       int32_t nseg, int64_t tiles, int32_t k, int32_t rule,
                                       int32_t trim_b, int64_t n, float* w, float* out, float lr,
                                       p2p_stream_t stream) {
  if (k < 1) return P2P_ERR_INVALID;
  if (k > 256) return P2P_ERR_UNSUPPORTED;
  if (rule == P2P_RULE_TRIMMED && (trim_b < 0 || k - 2 * trim_b <= 0)) return P2P_ERR_INVALID;
  if (rule != P2P_RULE_MEDIAN && rule != P2P_RULE_TRIMMED) return P2P_ERR_INVALID;
  RobustArgs a{peers, segs, nseg, tiles, k, trim_b, n, w, out, lr, static_cast<hipStream_t>(stream)};
  if (rule == P2P_RULE_MEDIAN) dispatch<P2P_RULE_MEDIAN>(a); else dispatch<P2P_RULE_TRIMMED>(a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? P2P_OK : static_cast<int32_t>(e);
}

extern "C" P2P_INTERNAL int64_t p2p_robust_tile_elems(void) { return kRobustTile; }
