// LAB (tools/, not built into the product): the pair scheme at K = 128 -- measured slower than the one-lane kernel (profiles/r02/ab128).
// K2 at K = 128 with the pruned rules (median; trimmed mean with b = 25):
// the two-wave pair scheme of robust_pair.hip at H = 64 keys per wave, two
// pairs per block so a block covers the one-lane kernels' 128-coordinate
// tile (segment tables keep one tile size per K).  Wave h of pair p loads
// peers 64h..64h+63 of coordinates c0 + 64p + lane, sorts them (Batcher
// sort64, float network unless the block holds a NaN), and the sorted halves
// meet in one flip through LDS exactly as at K = 256 (robust_pair.hip has the
// derivation); trimmed ranks 25..102 = 25..63 of L and 0..38 of U.  Against
// the one-lane kernel (robust.hip: a pruned 128-key network on uint32 keys)
// no key map, and ~100 VGPRs per wave instead of 147 / 155.
#include "robust_nets.h"

namespace p2p {
namespace pair128 {

// H = peers per wave (half of K): 128 for K = 256 (one pair per block, 64
// coordinates), 64 for K = 128 (two pairs per block, 128 coordinates -- the
// tile of the one-lane kernels, so segment tables keep one tile size per K).

__device__ __forceinline__ float val(fk x) { return x.x; }
__device__ __forceinline__ uint32_t raw(fk x) { return __float_as_uint(x.x); }
__device__ __forceinline__ uint32_t raw(uint32_t k) { return k; }
__device__ __forceinline__ float val(uint32_t k) { return __uint_as_float(key2f(k)); }
template <typename T> __device__ __forceinline__ T from_bits(uint32_t b);
template <> __device__ __forceinline__ fk from_bits<fk>(uint32_t b) { return fk{__uint_as_float(b)}; }
template <> __device__ __forceinline__ uint32_t from_bits<uint32_t>(uint32_t b) { return f2key(b); }
// An element as it crosses LDS: the T-domain word itself (float bits or key).
template <typename T> __device__ __forceinline__ T from_raw(uint32_t b);
template <> __device__ __forceinline__ fk from_raw<fk>(uint32_t b) { return fk{__uint_as_float(b)}; }
template <> __device__ __forceinline__ uint32_t from_raw<uint32_t>(uint32_t b) { return b; }

// LDS image of one sorted half: element j of lane l at word (j & 3) of
// slot [j >> 2][l] -- 1 KiB per ds_write_b128 / ds_read_b128, no bank conflict.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// Image slots read ahead of their use: the compiler would otherwise issue all
// 32 reads at once (and hold the other half in 128 more VGPRs).  fence_after
// makes a result computed from the slots read so far an input of a
// memory-clobbering asm, so neither that arithmetic sinks below nor later
// reads rise above it.
constexpr int kReadAhead = 4;
template <typename T>
__device__ __forceinline__ void fence_after(T& x) {
  uint32_t r = raw(x);
  asm volatile("" : "+v"(r)::"memory");
  x = from_raw<T>(r);
}
using Img = u32x4 __attribute__((address_space(3)))*;

__device__ __forceinline__ uint32_t img_at(Img im, int j, int lane) { return im[(j >> 2) * 64 + lane][j & 3]; }
template <int H> constexpr int img_slots() { return H / 4 * 64 + 16; }  // the image + 64 partial sums

// A wave-uniform flag the compiler also KNOWS is uniform: an inline-asm SGPR
// result counts as divergent, and a branch on it is linearised -- both the
// float and the key network then run under exec masks with the inputs live
// across both (376 VGPRs instead of ~200).
__device__ __forceinline__ bool uniform(bool x) {
  return __builtin_amdgcn_readfirstlane(static_cast<int>(x)) != 0;
}

template <int H, typename T>
__device__ __forceinline__ void store_half(Img im, const T (&x)[H], int lane) {
#pragma unroll
  for (int g = 0; g < H / 4; ++g)
    im[g * 64 + lane] = u32x4{raw(x[4 * g]), raw(x[4 * g + 1]), raw(x[4 * g + 2]), raw(x[4 * g + 3])};
}

// median: max_j min(B_j, A_{127-j}), A read from the image in T's domain.
template <int H, typename T>
__device__ __forceinline__ float median_final(Img im, const T (&b)[H], int lane) {
  T m{};
#pragma unroll
  for (int g = 0; g < H / 4; ++g) {
    const u32x4 a4 = im[(H / 4 - 1 - g) * 64 + lane];  // A_{127-4g-k} = word 3-k
    const T l0 = min(b[4 * g], from_raw<T>(a4[3])), l1 = min(b[4 * g + 1], from_raw<T>(a4[2]));
    const T l2 = min(b[4 * g + 2], from_raw<T>(a4[1])), l3 = min(b[4 * g + 3], from_raw<T>(a4[0]));
    const T q = max(max(l0, l1), max(l2, l3));
    m = g == 0 ? q : max(m, q);
    if (g % kReadAhead == kReadAhead - 1) fence_after(m);  // bound the reads in flight
  }
  return val(m);
}

// trimmed, wave 1: L_j = min(B_j, A_{127-j}) stays in b; U_j = max(...) is
// written over A_{127-j}'s word (each slot is read before it is rewritten).
template <int H, typename T>
__device__ __forceinline__ void flip_write_upper(Img im, T (&b)[H], int lane) {
#pragma unroll
  for (int g = 0; g < H / 4; ++g) {
    const int s = (H / 4 - 1 - g) * 64 + lane;
    const u32x4 a4 = im[s];
    u32x4 u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const T a = from_raw<T>(a4[3 - k]);
      const T lo = min(b[4 * g + k], a), hi = max(b[4 * g + k], a);
      b[4 * g + k] = lo;
      u[3 - k] = raw(hi);
    }
    im[s] = u;
    if (g % kReadAhead == kReadAhead - 1) fence_after(b[4 * g + 3]);
  }
}

// Sum of ranks [R0, R1) of a merged half, ascending, continuing from acc.
template <int R0, int R1, int H, typename T>
__device__ __forceinline__ float sum_ranks(const T (&x)[H], float acc) {
#pragma unroll
  for (int j = R0; j < R1; ++j) acc = __fadd_rn(acc, val(x[j]));
  return acc;
}

__device__ __forceinline__ void block_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Pins a sorted half where it is computed.  Without a use on both sides of
// the role branches LLVM sinks the network into one successor piecemeal, which
// scrambles its order (a 128-key sort then holds ~250 VGPRs instead of ~135).
template <int H, typename T>
__device__ __forceinline__ void pin(const T (&x)[H]) {
#pragma unroll
  for (int j = 0; j < H; ++j) asm volatile("" ::"v"(raw(x[j])));
}

// One half sorted in T's domain (the block's: keys if either half holds a
// NaN); returns the aggregate, valid where `own`.  Both waves pass the same
// number of block barriers.
template <int RULE, int H, int PAIRS>
__device__ __attribute__((noinline)) float pair_keys(const float* const* P, int64_t c0, uint32_t lane_off, Img im,
                                                     int h, int lane);

// FLAGS (float path): the two waves swap "my half holds a NaN" at barrier 1,
// beside the hand-off; a block that finds one re-runs the tile on the key
// network (pair_keys) -- the float sort of a NaN half is discarded.
template <int RULE, int H, int PAIRS, typename T, bool FLAGS = false>
__device__ __forceinline__ float pair_body(const uint32_t (&v)[H], Img im, int h, int lane,
                                           int __attribute__((address_space(3)))* flags = nullptr, bool nan = false,
                                           const float* const* P = nullptr, int64_t c0 = 0, uint32_t lane_off = 0) {
  T x[H];
#pragma unroll
  for (int j = 0; j < H; ++j) x[j] = from_bits<T>(v[j]);
  sort_full<H>(x);
  pin(x);
  if (h == 0) store_half(im, x, lane);
  if constexpr (FLAGS) {
    if (lane == 0) flags[0] = nan ? 1 : 0;  // this wave's flag
  }
  block_sync();  // 1: A in the image
  if constexpr (FLAGS) {  // one decision for the whole block: every pair passes the same barriers
    const int __attribute__((address_space(3)))* all = flags - (tid_x() >> 6);
    int any = 0;
#pragma unroll
    for (int q = 0; q < 2 * PAIRS; ++q) any |= all[q];
    if (uniform(any != 0)) return pair_keys<RULE, H, PAIRS>(P, c0, lane_off, im, h, lane);
  }
  if constexpr (RULE == P2P_RULE_MEDIAN) {
    return h == 1 ? median_final(im, x, lane) : 0.f;
  } else {
    constexpr int b = (2 * H * 2) / 10;  // 51 (K = 256) / 25 (K = 128)
    constexpr int hi = 2 * H - b;        // ranks b..hi-1 kept
    // the partial sum has a slot of its own past the image (no barrier
    // between wave 0's reads of U and wave 1's write of the partial)
    auto part = (float __attribute__((address_space(3)))*)(im + H / 4 * 64);
    if (h == 1) {
      flip_write_upper(im, x, lane);
      block_sync();  // 2: U_j in A_{127-j}'s word
      if constexpr (H == 128) net_bmerge128_r51_127<true>(x); else net_bmerge64_r25_63<true>(x);
      part[lane] = sum_ranks<b, H>(x, 0.f);
      block_sync();  // 3: the partial sum of ranks 51..127 in its slot
      return 0.f;
    }
    block_sync();  // 2
#pragma unroll
    for (int j = 0; j < H; ++j) x[j] = from_raw<T>(img_at(im, H - 1 - j, lane));
    if constexpr (H == 128) net_bmerge128_r0_76<true>(x); else net_bmerge64_r0_38<true>(x);
    block_sync();  // 3
    return sum_ranks<0, hi - H>(x, part[lane]) / static_cast<float>(hi - b);
  }
}

// This wave's 128 inputs of the tile.  Every load is the saddr form: the
// peer row's base plus the tile start in SGPRs, one 32-bit lane offset shared
// by all 128 loads -- no 64-bit VGPR address per load.  The asm keeps LLVM
// from re-associating the tile start into the lane offset.
template <int H>
__device__ __forceinline__ void load_half(uint32_t (&v)[H], const float* const* P, int64_t c0,
                                          uint32_t lane_off, int h) {
#pragma unroll
  for (int j = 0; j < H; ++j) {
    uint64_t row = reinterpret_cast<uint64_t>(table_at(P, h * H + j) + c0);
    asm("" : "+s"(row));
    v[j] = __float_as_uint(__builtin_nontemporal_load(
        reinterpret_cast<const P2P_GLOBAL float*>(reinterpret_cast<const P2P_GLOBAL char*>(row) + lane_off)));
  }
  __builtin_amdgcn_sched_barrier(0);  // all loads in flight before the first use
}

// The uint32-key network for a block holding a NaN.  Out of line and
// re-loading its inputs, so the float path's 128 values are not also held
// live for this one (inlined, the two paths took 320-390 VGPRs).
template <int RULE, int H, int PAIRS>
__device__ __attribute__((noinline)) float pair_keys(const float* const* P, int64_t c0, uint32_t lane_off, Img im,
                                                     int h, int lane) {
  // arguments arrive in VGPRs: make the wave-uniform ones scalar again
  P = reinterpret_cast<const float* const*>(uniform_u64(reinterpret_cast<uint64_t>(P)));
  c0 = static_cast<int64_t>(uniform_u64(static_cast<uint64_t>(c0)));
  h = __builtin_amdgcn_readfirstlane(h);
  uint32_t v[H];
  load_half<H>(v, P, c0, lane_off, h);
  return pair_body<RULE, H, PAIRS, uint32_t>(v, im, h, lane);
}

template <int RULE, bool SEGS, int H, int PAIRS>
__global__ __launch_bounds__(128 * PAIRS) __attribute__((amdgpu_waves_per_eu(3))) void robust_pair_kernel(
    const float* const* __restrict__ peers, const Seg* __restrict__ segs, int nseg, int64_t n, float* w, float* out,
    float lr) {
  constexpr int TILE = 64 * PAIRS;
  __shared__ u32x4 img_raw[PAIRS * img_slots<H>()];  // per pair: the image + 64 partial sums
  __shared__ int nan_flag[2 * PAIRS];
  const int wi = __builtin_amdgcn_readfirstlane(static_cast<int>(tid_x() >> 6));
  const int h = wi & 1, pr = wi >> 1;
  const int lane = tid_x() & 63;
  Img im = (Img)img_raw + pr * img_slots<H>();
  const int64_t t = bid_x();
  const float* const* P = peers;
  float* W = w;
  float* O = out;
  int64_t N = n, c0 = t * TILE;
  if constexpr (SEGS) {
    const Seg s = load_segment(segs, nseg, t);
    P = s.peers;
    W = s.w;
    O = s.out;
    N = s.n;
    c0 = (t - s.tile_begin) * TILE;
  }
  c0 += 64 * pr;  // this pair's 64 coordinates
  const int64_t i = c0 + lane;
  // Dead lanes of a ragged tail re-read the last element (a pair wholly past
  // the end re-reads it too: every wave must reach the block's barriers).
  const int64_t ic = i < N ? i : N - 1;
  const uint32_t lane_off = static_cast<uint32_t>(ic - (c0 < N ? c0 : N - 1)) * 4u;
  const int64_t cb = c0 < N ? c0 : N - 1;  // row base of this pair
  uint32_t v[H];
  load_half<H>(v, P, cb, lane_off, h);
  // One domain per block: the float network unless any half holds a NaN
  // (flags swapped at the hand-off barrier, no barrier of their own).
  const bool nan = uniform(wave_has_nan(v));
  const float agg = pair_body<RULE, H, PAIRS, fk, true>(
      v, im, h, lane, (int __attribute__((address_space(3)))*)nan_flag + wi, nan, P, cb, lane_off);
  const bool own = RULE == P2P_RULE_MEDIAN ? h == 1 : h == 0;
  if (own && i < N) {
    if (O) stg(O + i, agg);
    if (W) stg(W + i, apply_lr(ldg(W + i), lr, agg));
  }
}

}  // namespace pair128

template <int H, int PAIRS>
static void launch_pair128(const float* const* peers, const p2p_segment_t* segs, int32_t nseg, int64_t tiles,
                        int32_t rule, int64_t n, float* w, float* out, float lr, hipStream_t st) {
  const int64_t grid = segs ? tiles : ceil_div(n, 64 * PAIRS);
  if (grid <= 0) return;
  const dim3 g(static_cast<unsigned>(grid)), b(128 * PAIRS);
  if (rule == P2P_RULE_MEDIAN) {
    if (segs) hipLaunchKernelGGL((pair128::robust_pair_kernel<P2P_RULE_MEDIAN, true, H, PAIRS>), g, b, 0, st, peers, segs, nseg, n, w, out, lr);
    else hipLaunchKernelGGL((pair128::robust_pair_kernel<P2P_RULE_MEDIAN, false, H, PAIRS>), g, b, 0, st, peers, segs, nseg, n, w, out, lr);
  } else {
    if (segs) hipLaunchKernelGGL((pair128::robust_pair_kernel<P2P_RULE_TRIMMED, true, H, PAIRS>), g, b, 0, st, peers, segs, nseg, n, w, out, lr);
    else hipLaunchKernelGGL((pair128::robust_pair_kernel<P2P_RULE_TRIMMED, false, H, PAIRS>), g, b, 0, st, peers, segs, nseg, n, w, out, lr);
  }
}

}  // namespace p2p

using namespace p2p;

// K = 128 (median, or trimmed with b = 25): 128-coordinate tiles of two pairs.
// Flat: ceil(n / 128) blocks; segment table: `tiles`, tile_begin in tiles.
extern "C" P2P_INTERNAL void p2p_robust_pair128_launch(const float* const* peers, const p2p_segment_t* segs,
                                                       int32_t nseg, int64_t tiles, int32_t rule, int64_t n,
                                                       float* w, float* out, float lr, p2p_stream_t stream) {
  launch_pair128<64, 2>(peers, segs, nseg, tiles, rule, n, w, out, lr, static_cast<hipStream_t>(stream));
}
