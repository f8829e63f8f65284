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
// K <= 128: ONE LANE per coordinate (KP = next power of two, +inf pads; a
// network pruned to the wanted ranks when K == KP in {64, 128}, and for any
// K in 33..127 padded at both ends of the order into those networks -- PAD).  The float
// network of robust_nets.h is NOT used here: holding the float copy next to
// the keys took the K = 128 kernels from 146 / 183 VGPRs (3 / 2 waves per
// SIMD) to 256 (1 wave) and cfg4 from 73% / 60% to 59% / 52% of HBM peak.  Loads:
// each wave instruction reads 256 contiguous bytes of one peer; all KP loads
// are issued before the first compare.  K in 129..256 is robust_lds.hip.
#include "robust_nets.h"

namespace p2p {

constexpr int kRobustTile = 128;  // coordinates per block (one lane each)

// PAD (round 4): K in KP/2+1..KP-1 (or another trim) runs the K == KP
// networks on KP slots, slots >= K being pads -- the first `lo` of them the
// bottom of the order (-inf / key 0), the rest the top (+inf / key ~0); every
// real key orders between them and ties are the same value.  Median:
// lo = (KP-1)/2 - (K-1)/2 puts the real lower median at rank (KP-1)/2, the
// four-list search's.  Trimmed: lo = b0 - b (b0 = floor(0.2 KP), the pruned
// network's) puts the kept real ranks b..K-b-1 at b0..b0+m-1 (m = K - 2b),
// summed while k < m.  robust_pad_fits says when the pads fit.  A pad slot
// loads from a pad row (robust_nets.h pad_row), so the networks and the NaN
// test see the pads with no select.
__host__ __device__ constexpr int pad_lo(int KP, int rule, int K, int trim_b) {
  return rule == P2P_RULE_MEDIAN ? (KP - 1) / 2 - (K - 1) / 2 : (KP * 2) / 10 - trim_b;
}

// K == KP: the pruned rules on the float values (robust_nets.h: same ranks and
// bits as the keys) -- no key map in (2 VALU per key) or out.  `nan` collects
// the NaN test block by block as the networks first read each block; the
// result is valid only when it stays 0.
template <int KP, int RULE, bool PAD = false>
__device__ __forceinline__ float special_floats(const uint32_t (&v)[KP], uint64_t& nan, int K = KP, int trim_b = 0) {
  auto at = [&](int j) { return __uint_as_float(v[j]); };
  if constexpr (RULE == P2P_RULE_MEDIAN) {
    constexpr int Q = KP / 4;
    fk a[Q], b[Q], c[Q], d[Q];
#pragma unroll
    for (int j = 0; j < Q; ++j) {
      a[j].x = at(j);
      b[j].x = at(Q + j);
      c[j].x = at(2 * Q + j);
      d[j].x = at(3 * Q + j);
    }
    // PAD: lists c and d (slots KP/2..KP-1) may hold pad rows
    constexpr int S = PAD ? 0 : 1 << 20;
    sort_full<Q>(a, NanHook<>{nan});
    sort_full<Q>(b, NanHook<>{nan});
    sort_full<Q>(c, NanHook<1, 0, S>{nan});
    sort_full<Q>(d, NanHook<1, 0, S>{nan});
    return four_list_median<Q>(a, b, c, d).x;
  } else {
    fx x[KP];
#pragma unroll
    for (int j = 0; j < KP; ++j) x[j].x = at(j);
    run_special<KP, 2>(x, NanHook<1, 0, PAD ? KP / 32 : 1 << 20>{nan});  // PAD: blocks of slots >= KP/2
    constexpr int b = (KP * 2) / 10;
    float acc = 0.f;
    if constexpr (PAD) {  // padded ranks b..b+m-1
      const int m = K - 2 * trim_b;
#pragma unroll
      for (int j = b; j < KP - b; ++j) {
        if (j - b < m) acc = __fadd_rn(acc, x[j].x);  // a uniform condition
      }
      return acc / static_cast<float>(m);
    }
#pragma unroll
    for (int j = b; j < KP - b; ++j) acc = __fadd_rn(acc, x[j].x);
    return div_const<KP - 2 * b>(acc);  // = acc / float(KP - 2b), bit for bit (robust_nets.h)
  }
}

template <int KP, int RULE, int MODE, bool PAD>
__device__ __attribute__((noinline)) float robust_coord_keys(const float* const* peers, int K, int trim_b,
                                                             int64_t c0, uint32_t lane_off);

// KEYS: the uint32 total-order key network (MODE 0, or a wave holding a NaN);
// otherwise (K == KP) the float network unless the wave holds a NaN, which
// re-runs on the keys out of line (re-loading: inlined, LLVM kept both
// paths' values live, 256 VGPRs and one wave per SIMD).
template <int KP, int RULE, int MODE, bool PAD = false, bool KEYS = MODE == 0>
__device__ __forceinline__ float robust_coord(const float* const* __restrict__ peers, int K,
                                              int trim_b, int64_t c0, uint32_t lane_off) {
  // Loads are unconditional (a pad slot re-reads peer 0, an L2 hit) so the
  // compiler can keep all of them in flight: a branch around each load made
  // it wait for every load before the branch merge (serialised, ~8x slower).
  // Each is the saddr form: the peer row's base + the tile start in SGPRs and
  // one 32-bit lane offset shared by every load (no 64-bit VGPR address per
  // load); the asm keeps LLVM from re-associating the tile start into it.
  uint32_t v[KP];
  const int lo = PAD ? pad_lo(KP, RULE, K, trim_b) : 0;
  const uint64_t prow = reinterpret_cast<uint64_t>(pad_row(KEYS, false));  // the top row follows it
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    const bool real = (MODE != 0 && !PAD) || (PAD && 2 * j < KP) || (j < K);  // PAD: K > KP / 2
    uint64_t row = reinterpret_cast<uint64_t>(table_at(peers, PAD ? min(j, K - 1) : real ? j : 0) + c0);
    // PAD: a pad slot reads its pad row (no c0: the row is one tile wide)
    if (PAD && !real) row = prow + (j - K >= lo ? kPadRowBytes : 0u);
    asm("" : "+s"(row));
    const P2P_GLOBAL float* src =
        reinterpret_cast<const P2P_GLOBAL float*>(reinterpret_cast<const P2P_GLOBAL char*>(row) + lane_off);
    // a slot that may be a pad loads through the caches (every wave of the
    // chip reads the same pad rows: streamed, they would all go to one L2
    // channel); peer rows stream
    v[j] = __float_as_uint(PAD && 2 * j >= KP ? *src : __builtin_nontemporal_load(src));
  }
  __builtin_amdgcn_sched_barrier(0);  // all KP loads in flight before the first use
  if constexpr (MODE != 0 && !KEYS) {  // K == KP: a NaN-free wave runs on the floats themselves
    uint64_t nan = 0;
    const float r = special_floats<KP, RULE, PAD>(v, nan, K, trim_b);
    if (!__builtin_amdgcn_readfirstlane(static_cast<int>(nan != 0))) return r;
    return robust_coord_keys<KP, RULE, MODE, PAD>(peers, K, trim_b, c0, lane_off);
  }
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    // MODE 0: a pad sorts after every real key; PAD: the pad row's bits map
    // to the bottom / top key
    const bool real = (MODE != 0) || (j < K);
    v[j] = real ? f2key(v[j]) : 0xFFFFFFFFu;
  }
  if constexpr (RULE == P2P_RULE_MEDIAN && MODE == 1) {
    // K == KP in {64, 128}: four sorted lists of KP/4 and the two-set search
    // (robust_nets.h) -- 1.9k VALU at K = 128 against 2.3k for the pruned
    // Batcher median network.
    constexpr int Q = KP / 4;
    uint32_t a[Q], b[Q], c[Q], d[Q];
#pragma unroll
    for (int j = 0; j < Q; ++j) {
      a[j] = v[j];
      b[j] = v[Q + j];
      c[j] = v[2 * Q + j];
      d[j] = v[3 * Q + j];
    }
    sort_full<Q>(a);
    sort_full<Q>(b);
    sort_full<Q>(c);
    sort_full<Q>(d);
    return __uint_as_float(key2f(four_list_median<Q>(a, b, c, d)));
  } else if constexpr (MODE == 0) {
    sort_full<KP>(v);
  } else if constexpr (RULE == P2P_RULE_TRIMMED && KP == 128) {  // fewer live VGPRs: 3 waves/SIMD
    kx x[KP];
#pragma unroll
    for (int j = 0; j < KP; ++j) x[j].k = v[j];
    run_special<KP, MODE>(x);
#pragma unroll
    for (int j = 0; j < KP; ++j) v[j] = x[j].k;
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
    if constexpr (MODE == 2 && PAD) {
      constexpr int b = (KP * 2) / 10;  // padded ranks b..b+m-1
      const int m = K - 2 * trim_b;
#pragma unroll
      for (int j = b; j < KP - b; ++j) {
        if (j - b < m) acc = __fadd_rn(acc, __uint_as_float(key2f(v[j])));  // a uniform condition
      }
      return acc / static_cast<float>(m);
    } else if constexpr (MODE == 2) {
      constexpr int b = (KP * 2) / 10;  // floor(0.2 KP) for KP in {64,128,256}
#pragma unroll
      for (int j = b; j < KP - b; ++j) acc = __fadd_rn(acc, __uint_as_float(key2f(v[j])));
      return div_const<KP - 2 * b>(acc);
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

template <int KP, int RULE, int MODE, bool PAD>
__device__ __attribute__((noinline)) float robust_coord_keys(const float* const* peers, int K, int trim_b,
                                                             int64_t c0, uint32_t lane_off) {
  // arguments arrive in VGPRs: make the wave-uniform ones scalar again
  peers = reinterpret_cast<const float* const*>(uniform_u64(reinterpret_cast<uint64_t>(peers)));
  c0 = static_cast<int64_t>(uniform_u64(static_cast<uint64_t>(c0)));
  K = __builtin_amdgcn_readfirstlane(K);
  trim_b = __builtin_amdgcn_readfirstlane(trim_b);
  return robust_coord<KP, RULE, MODE, PAD, true>(peers, K, trim_b, c0, lane_off);
}

// ---- kernels ---------------------------------------------------------------
// KP <= 128 (template arg): one lane per coordinate, 128-lane blocks.
// P in {2, 4} (GROUP kernels): 128*P-lane blocks.  A block covers kRobustTile
// coordinates either way.
template <int KP, int RULE, int MODE, bool PAD>
__device__ __forceinline__ void robust_one(const float* const* peers, int K, int trim_b, int64_t n,
                                           int64_t tile, float* w, float* out, float lr) {
  const int64_t c0 = tile * kRobustTile;
  const int64_t i = c0 + tid_x();
  if (i >= n) return;
  const float agg = robust_coord<KP, RULE, MODE, PAD>(peers, K, trim_b, c0, tid_x() * 4u);
#if P2P_ROBUST_STORE_AUX < 0
  if (out) stg(out + i, agg);
  if (w) stg(w + i, apply_lr(ldg(w + i), lr, agg));
#else
  // descriptors at the tile's base (wave-uniform), the lane's float at tid * 4
  if (out) {
    float* ob = reinterpret_cast<float*>(uniform_u64(reinterpret_cast<uint64_t>(out + c0)));
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(agg), __builtin_amdgcn_make_buffer_rsrc(ob, 0, kRobustTile * 4, 0x00020000),
                                          tid_x() * 4u, 0, P2P_ROBUST_STORE_AUX);
  }
  if (w) {
    float* wb = reinterpret_cast<float*>(uniform_u64(reinterpret_cast<uint64_t>(w + c0)));
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(apply_lr(ldg(w + i), lr, agg)),
                                          __builtin_amdgcn_make_buffer_rsrc(wb, 0, kRobustTile * 4, 0x00020000),
                                          tid_x() * 4u, 0, P2P_ROBUST_STORE_AUX);
  }
#endif
}

// 2-D grid (p2p_common.h tile_grid): tile t = blockIdx.y * gx + blockIdx.x.
template <int KP, int RULE, int MODE, bool PAD>
__global__ __launch_bounds__(kRobustTile, MODE != 0 ? 3 : 1) void robust_flat_kernel(
    const float* const* __restrict__ peers, int K, int trim_b, int64_t n, float* w, float* out,
    float lr, int64_t ntiles, unsigned gx) {
  const int64_t t = tile_id(gx);
  if (t >= ntiles) return;
  robust_one<KP, RULE, MODE, PAD>(peers, K, trim_b, n, t, w, out, lr);
}

template <int KP, int RULE, int MODE, bool PAD>
__global__ __launch_bounds__(kRobustTile, MODE != 0 ? 3 : 1) void robust_segments_kernel(
    const Seg* __restrict__ segs, int nseg, int K, int trim_b, float lr, int64_t ntiles, unsigned gx) {
  const int64_t t = tile_id(gx);
  if (t >= ntiles) return;
  const Seg s = load_segment(segs, nseg, t);
  robust_one<KP, RULE, MODE, PAD>(s.peers, K, trim_b, s.n, t - s.tile_begin, s.w, s.out, lr);
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

template <int KP, int RULE, int MODE, bool PAD = false>
static void launch_one(const RobustArgs& a) {
  const int64_t tiles = a.segs ? a.tiles : ceil_div(a.n, kRobustTile);
  const TileGrid g = tile_grid(tiles, kRobustTile);
  if (g.gx == 0) return;
  if (a.segs) {
    hipLaunchKernelGGL((robust_segments_kernel<KP, RULE, MODE, PAD>), dim3(g.gx, g.gy), dim3(kRobustTile), 0, a.stream,
                       a.segs, a.nseg, a.K, a.trim_b, a.lr, tiles, g.gx);
  } else {
    hipLaunchKernelGGL((robust_flat_kernel<KP, RULE, MODE, PAD>), dim3(g.gx, g.gy), dim3(kRobustTile), 0, a.stream,
                       a.peers, a.K, a.trim_b, a.n, a.w, a.out, a.lr, tiles, g.gx);
  }
}

// The pads fit a K < KP (or another trim) into the K == KP networks: the
// median always; the trimmed mean while b <= b0, K - b <= KP - b0 and
// m = K - 2b <= KP - 2 b0 (every K in 33..128 at the default 0.2 trim).
static bool robust_pad_fits(int KP, int rule, int K, int b) {
  if (K > KP || 2 * K <= KP) return false;
  if (rule == P2P_RULE_MEDIAN) return true;
  const int b0 = (KP * 2) / 10;
  return b >= 0 && b <= b0 && K - b <= KP - b0 && K - 2 * b >= 1 && K - 2 * b <= KP - 2 * b0;
}

template <int KP, int RULE>
static void launch_kp(const RobustArgs& a) {
  if constexpr (KP == 64 || KP == 128) {
    constexpr int MODE = RULE == P2P_RULE_MEDIAN ? 1 : 2;
    if (a.K == KP && (RULE == P2P_RULE_MEDIAN || a.trim_b == (KP * 2) / 10)) return launch_one<KP, RULE, MODE>(a);
    if (robust_pad_fits(KP, RULE, a.K, a.trim_b)) return launch_one<KP, RULE, MODE, true>(a);
  }
  launch_one<KP, RULE, 0>(a);
}

// Layout per (rule, K), from measurements on MI355X:
//   K <= 128     one lane per coordinate, this file (cfg4: median 64-71%,
//                trimmed 54% of HBM peak at K = 128)
//   K 129..256   4 lanes x 64 keys per coordinate, peer rows LDS-DMA staged
//                (robust_lds.hip)
// The layouts measured slower (wave groups exchanging through LDS, LDS
// staging for K <= 128, 2 x 64 / 1 x 128 keys per lane) are kept out of the
// product library; tools/robust_lab.hip rebuilds them for A/B runs.
template <int RULE>
static void dispatch(const RobustArgs& a) {
  if (a.K <= 2) return launch_kp<2, RULE>(a);
  if (a.K <= 4) return launch_kp<4, RULE>(a);
  if (a.K <= 8) return launch_kp<8, RULE>(a);
  if (a.K <= 16) return launch_kp<16, RULE>(a);
  if (a.K <= 32) return launch_kp<32, RULE>(a);
  if (a.K <= 64) return launch_kp<64, RULE>(a);
  launch_kp<128, RULE>(a);
}

}  // namespace p2p

using namespace p2p;

extern "C" P2P_INTERNAL int64_t p2p_robust_lds_tile(int32_t rule, int32_t k);
extern "C" P2P_INTERNAL void p2p_robust_lds_launch(const float* const* peers, const p2p_segment_t* segs,
                                                   int32_t nseg, int64_t tiles, int32_t k, int32_t rule,
                                                   int32_t trim_b, int64_t n, float* w, float* out, float lr,
                                                   p2p_stream_t stream);

// Stateless: the kernel family and its tile size are pure functions of (rule, k).
extern "C" P2P_INTERNAL int32_t p2p_robust_dispatch(const float* const* peers, const p2p_segment_t* segs,
                                                    int32_t nseg, int64_t tiles, int32_t k, int32_t rule,
                                                    int32_t trim_b, int64_t n, float* w, float* out, float lr,
                                                    p2p_stream_t stream) {
  if (k < 1) return P2P_ERR_INVALID;
  if (k > 256) return P2P_ERR_UNSUPPORTED;
  if (rule == P2P_RULE_TRIMMED && (trim_b < 0 || k - 2 * trim_b <= 0)) return P2P_ERR_INVALID;
  if (rule != P2P_RULE_MEDIAN && rule != P2P_RULE_TRIMMED) return P2P_ERR_INVALID;
  if (k > 128) {
    p2p_robust_lds_launch(peers, segs, nseg, tiles, k, rule, trim_b, n, w, out, lr, stream);
  } else {
    RobustArgs a{peers, segs, nseg, tiles, k, trim_b, n, w, out, lr, static_cast<hipStream_t>(stream)};
    if (rule == P2P_RULE_MEDIAN) dispatch<P2P_RULE_MEDIAN>(a); else dispatch<P2P_RULE_TRIMMED>(a);
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? P2P_OK : static_cast<int32_t>(e);
}

extern "C" P2P_INTERNAL int64_t p2p_robust_tile_elems(int32_t rule, int32_t k) {
  return k > 128 ? p2p_robust_lds_tile(rule, k) : kRobustTile;
}
