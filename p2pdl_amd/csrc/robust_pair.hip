// K2 at K = 256 with the pruned rules (median; trimmed mean with b = 51):
// ONE lane per coordinate, a block of two waves over 64 coordinates.
//
// Rule (no reference implementation, README.md:10):
//   median : key of rank 127 under the IEEE total order on float bits
//   trimmed: fp32 sum of ranks 51..204 ascending from +0, IEEE-divided by 154
// then w += lr*agg, multiply and add separately rounded (aggregation.py:36-38).
//
// Wave h loads peers 128h..128h+127 of its 64 coordinates (every load
// instruction reads 256 contiguous bytes of one peer) -- half A (h = 0) and
// half B (h = 1).
//   median : each wave sorts its half as two lists of 64 and the two-set
//            search (robust_nets.h) finds rank 127 without merging them.
//   trimmed: each wave sorts its 128 (Batcher, three-input lowered) and the
//            two halves meet in Batcher's odd-even merge split by parity:
//            v = merge(A_even, B_even) in wave 0, w = merge(A_odd, B_odd) in
//            wave 1 (each hands the other parity over, 16 KB), pruned to the
//            ranks that reach 51..204 (398 instructions each); the merged
//            order is c_{2i-1} = min(v_i, w_{i-1}), c_{2i} = max(v_i, w_{i-1}),
//            so 39 values cross per wave, wave 1 sums c_51..c_127 ascending
//            and wave 0 carries on over c_128..c_204 (the partial crosses LDS
//            through a slot of its own).  Against the round-2 flip + pruned
//            bitonic mergers: 475 instead of 558 instructions per wave.
// Against the 4-lanes-per-coordinate LDS kernel this issues ~10% (median) /
// ~22% (trimmed) fewer VALU instructions per coordinate -- two 128-key sorts
// instead of four 64-key sorts plus cross-lane bitonic merges, no DPP moves,
// and the trimmed sum advances 64 coordinates per instruction instead of 16 --
// and no wave only loads: every wave sorts, 2 per SIMD (<= 256 VGPRs; 32 KB of
// LDS per block, 4 blocks per CU), each hiding the other's HBM latency.
//
// Float or key network, per block: each wave sorts its half on the float
// values themselves (robust_nets.h: same order, same bits as the uint32
// keys), and the waves learn at the hand-off barrier whether either half
// holds a NaN (median: a flag per wave; trimmed: each other's rank-0
// output, which every NaN reaches); a block that finds one re-runs the tile
// on uint32 total-order keys.  That key path is out of line and re-loads its inputs (pair_keys):
// inlined next to the float path, LLVM kept both paths' 128 values live and
// the kernel took 320-390 VGPRs.
#include "robust_nets.h"

namespace p2p {

constexpr int kPairTile = 64;  // coordinates per wave pair, one lane each
// Wave pairs per block: the median kernel runs two pairs on adjacent 64-
// coordinate tiles, so each peer row is read 512 contiguous bytes per block
// (two 256-B wave loads issued together) instead of 256.
constexpr int kMedianPairs = 2;
constexpr int kTrimPairs = 1;  // the trimmed mean's pair and LDS kernels share the 64-coordinate tile
constexpr int kHalf = 128;     // peers per wave

__device__ __forceinline__ float val(fk x) { return x.x; }
__device__ __forceinline__ uint32_t raw(fk x) { return __float_as_uint(x.x); }
__device__ __forceinline__ uint32_t raw(uint32_t k) { return k; }
__device__ __forceinline__ float val(uint32_t k) { return __uint_as_float(key2f(k)); }
__device__ __forceinline__ uint32_t raw(kx k) { return k.k; }
__device__ __forceinline__ float val(kx k) { return __uint_as_float(key2f(k.k)); }
template <typename T> __device__ __forceinline__ T from_bits(uint32_t b);
template <> __device__ __forceinline__ fk from_bits<fk>(uint32_t b) { return fk{__uint_as_float(b)}; }
template <> __device__ __forceinline__ uint32_t from_bits<uint32_t>(uint32_t b) { return f2key(b); }
template <> __device__ __forceinline__ kx from_bits<kx>(uint32_t b) { return kx{f2key(b)}; }
// An element as it crosses LDS: the T-domain word itself (float bits or key).
template <typename T> __device__ __forceinline__ T from_raw(uint32_t b);
template <> __device__ __forceinline__ fk from_raw<fk>(uint32_t b) { return fk{__uint_as_float(b)}; }
template <> __device__ __forceinline__ uint32_t from_raw<uint32_t>(uint32_t b) { return b; }
template <> __device__ __forceinline__ kx from_raw<kx>(uint32_t b) { return kx{b}; }

// LDS image of one sorted half: element j of lane l at word (j & 3) of
// slot [j >> 2][l] -- 1 KiB per ds_write_b128 / ds_read_b128, no bank conflict.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
using Img = u32x4 __attribute__((address_space(3)))*;

__device__ __forceinline__ uint32_t img_at(Img im, int j, int lane) { return im[(j >> 2) * 64 + lane][j & 3]; }

// A wave-uniform flag the compiler also KNOWS is uniform: an inline-asm SGPR
// result counts as divergent, and a branch on it is linearised -- both the
// float and the key network then run under exec masks with the inputs live
// across both (376 VGPRs instead of ~200).
__device__ __forceinline__ bool uniform(bool x) {
  return __builtin_amdgcn_readfirstlane(static_cast<int>(x)) != 0;
}

template <typename T>
__device__ __forceinline__ void store_half(Img im, const T (&x)[kHalf], int lane) {
#pragma unroll
  for (int g = 0; g < kHalf / 4; ++g)
    im[g * 64 + lane] = u32x4{raw(x[4 * g]), raw(x[4 * g + 1]), raw(x[4 * g + 2]), raw(x[4 * g + 3])};
}

// Word image of the trimmed path: element j of lane l at word j*64 + l.  A
// pair of rows is one ds_write2st64_b32 / ds_read2st64_b32 from / into ANY
// two VGPRs, conflict-free -- the b128 image needs its 4 words in consecutive
// VGPRs, and a network's outputs are not: 64 v_mov per wave on the hand-off.
using W32 = uint32_t __attribute__((address_space(3)))*;

__device__ __forceinline__ uint32_t row_at(W32 im, int j, int lane) { return im[j * 64 + lane]; }

// m[FIRST .. FIRST+N-1] as rows 0..N-1 of a word image.
template <int FIRST, int N, typename T>
__device__ __forceinline__ void send_run(W32 dst, const T (&m)[kHalf], int lane) {
#pragma unroll
  for (int j = 0; j < N; ++j) dst[j * 64 + lane] = raw(m[FIRST + j]);
}

// A raw buffer descriptor over a flat float buffer (stride 0, byte offsets;
// dword 3 as gfx9 parts take it).  An access past num_records reads 0 /
// drops the store, so the range is the whole 32-bit byte space: NARROW
// buffers (kNarrowMaxN below) keep every live lane's last byte under it --
// the round-5 descriptor's 2^31 - 1 silently dropped coordinates >= 2^29.
constexpr uint32_t kRsrcBytes = 0xFFFFFFFFu;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t flat_rsrc(float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, kRsrcBytes, 0x00020000);
}
// Largest flat n the NARROW path takes: a lane's 32-bit byte offset
// (c0 + lane) * 4 -- c0 + lane <= n - 1 + 63 -- must neither wrap nor leave
// the descriptor's range with its 4-byte access.
constexpr int64_t kNarrowMaxN = (int64_t(1) << 30) - 1024;
static_assert((kNarrowMaxN - 1 + 63) * 4 + 4 <= int64_t(kRsrcBytes), "NARROW offsets inside the descriptor");

__device__ __forceinline__ void block_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Pins a sorted half where it is computed.  Without a use on both sides of
// the role branches LLVM sinks the network into one successor piecemeal, which
// scrambles its order (a 128-key sort then holds ~250 VGPRs instead of ~135).
template <int N, typename T>
__device__ __forceinline__ void pin(const T (&x)[N]) {
#pragma unroll
  for (int j = 0; j < N; ++j) asm volatile("" ::"v"(raw(x[j])));
}

// K in 129..255 (PAD kernels): the block sorts a padded 256 -- wave h holds
// slots 128h..128h+127, slots >= K are pads, the first `lo` of them at the
// bottom of the order and the rest at the top (+-inf on the float path,
// keys 0 / ~0 on the key path: every real key orders between them, ties
// are the same value).  The median takes lo = 127 - (K-1)/2, so rank 127 of
// the 256 is the real lower median; the trimmed mean lo = 51 - b, so the
// kept real ranks b..K-b-1 are padded ranks 51..51+m-1 (m = K - 2b <= 154)
// and the sum stops after m of them.  A pad slot loads its word from a pad
// row (robust_nets.h pad_row: the row is one tile wide, so the PAD kernels
// keep the tile start in the row base, not in the lane offset).
struct Pads {
  int lo = 0;      // low pads
  int m = 2 * kHalf - 2 * 51;  // trimmed: kept ranks
};

// One half sorted in T's domain (the block's: keys if either half holds a
// NaN); returns the aggregate, valid in wave 0.  Both waves pass the same
// number of block barriers.
template <int RULE, bool PAD>
__device__ __attribute__((noinline)) float pair_keys(const float* const* P, int64_t c0, uint32_t lane_off, Img im,
                                                     int h, int lane, int K, int lo, int m);

// MEDIAN (rank 127 of 256) without sorting the halves: wave h sorts its
// peers as two lists of 64 (p = peers 128h..128h+63, q = the next 64) and
// splits its 128 by one flip, lo_j = min(p_j, q_{63-j}) (the 64 smallest,
// bitonic) / hi_j = max(...).  The waves swap max(lo) (barrier 1) and both
// make the same choice: A_hi u B_lo if max(A_lo) <= max(B_lo), else
// A_lo u B_hi.  Wave 1 builds its half of that choice as one v_med3 per key
// and hands it over (16 KB, barrier 2); wave 0 builds its own and runs the
// two-set search (robust_nets.h).  Against two Batcher sorts of 128 and the
// flip this issues 17% fewer VALU instructions per coordinate; the 16 KB
// image leaves room for 3 blocks' worth of waves per SIMD pair.
template <typename T, bool FLAGS = false, bool PAD = false, int NP = 1>
__device__ __forceinline__ float median_pair(const uint32_t (&v)[kHalf], Img im, int h, int lane,
                                             int __attribute__((address_space(3)))* flags = nullptr,
                                             const float* const* P = nullptr, int64_t c0 = 0, uint32_t lane_off = 0,
                                             int K = 2 * kHalf, const Pads& pd = Pads{}, int pr = 0) {
  constexpr int Q = kHalf / 2;  // 64 keys per sorted list
  // FLAGS: the NaN test is one compare of each sort's rank-0 output: every
  // min in its cone propagates NaN (gen_networks.py NAN_CONE_TAGS), so a NaN
  // among a list's 64 keys reaches p[0] / q[0]
  T p[Q], q[Q];
#pragma unroll
  for (int j = 0; j < Q; ++j) p[j] = from_bits<T>(v[j]);
  sort_full<Q>(p);
#pragma unroll
  for (int j = 0; j < Q; ++j) q[j] = from_bits<T>(v[Q + j]);
  sort_full<Q>(q);
  uint64_t nan = 0;
  if constexpr (FLAGS) nan = unordered_mask(bits_f(p[0]), bits_f(q[0]));
  const bool has_nan = FLAGS && uniform(nan != 0);  // to a bool at once (a live mask spilled SGPRs)
  pin(p);
  pin(q);
  // max_j min(p_j, q_{63-j}) as a v_max3 chain (the mins consumed as made)
  T m = min(p[0], q[Q - 1]);
#pragma unroll
  for (int j = 1; j + 1 < Q; j += 2) m = max(max(m, min(p[j], q[Q - 1 - j])), min(p[j + 1], q[Q - 2 - j]));
  m = max(m, min(p[Q - 1], q[0]));
  auto part = (uint32_t __attribute__((address_space(3)))*)(im + Q / 4 * 64);  // max(lo) of wave h at [64h + lane]
  part[h * 64 + lane] = raw(m);
  if constexpr (FLAGS) {
    if (lane == 0) flags[2 * pr + h] = has_nan ? 1 : 0;
  }
  block_sync();  // 1: both max(lo)
  if constexpr (FLAGS) {  // block-wide: every pair of the block takes the same path (same barriers)
    if (uniform((flags[0] | flags[1] | (NP > 1 ? flags[2] | flags[3] : 0) | (NP > 2 ? flags[4] | flags[5] : 0)) != 0))
      return pair_keys<P2P_RULE_MEDIAN, PAD>(P, c0, lane_off, im, h, lane, K, pd.lo, pd.m);
  }
  const T mo = from_raw<T>(part[(1 - h) * 64 + lane]);
  const bool d = h == 0 ? le(m, mo) : le(mo, m);  // max(A_lo) <= max(B_lo): A_hi u B_lo
  // wave 0 keeps A_hi (d) / A_lo; wave 1 keeps B_lo (d) / B_hi: the top limit iff d == (h == 0)
  const T lim = keep_limit(T{}, d == (h == 0));
  T x[Q];
#pragma unroll
  for (int j = 0; j < Q; ++j) x[j] = keep(p[j], q[Q - 1 - j], lim);
  if (h == 1) {
#pragma unroll
    for (int g = 0; g < Q / 4; ++g) im[g * 64 + lane] = u32x4{raw(x[4 * g]), raw(x[4 * g + 1]), raw(x[4 * g + 2]), raw(x[4 * g + 3])};
  }
  block_sync();  // 2: B's kept half in the image
  if (h == 1) return 0.f;
  T y[Q];
#pragma unroll
  for (int j = 0; j < Q; ++j) y[j] = from_raw<T>(img_at(im, j, lane));
  return val(two_set_median<Q>(x, y));
}

// FLAGS (float path): the two waves learn at barrier 1, beside the hand-off,
// whether either half holds a NaN; a block that finds one re-runs the tile
// on the key network (pair_keys) -- the float sort of a NaN half is
// discarded.  NP == 1 (the product's trimmed kernels) reports it through
// *redo and the caller re-runs after the float path; NP > 1 calls here.
template <int RULE, typename T, bool FLAGS = false, bool PAD = false, int NP = 1>
__device__ __forceinline__ float pair_body(const uint32_t (&v)[kHalf], Img im, int h, int lane,
                                           int __attribute__((address_space(3)))* flags = nullptr,
                                           const float* const* P = nullptr, int64_t c0 = 0, uint32_t lane_off = 0,
                                           int K = 2 * kHalf, const Pads& pd = Pads{}, int pr = 0,
                                           bool* redo = nullptr) {
  T x[kHalf];
#pragma unroll
  for (int j = 0; j < kHalf; ++j) x[j] = from_bits<T>(v[j]);
  // FLAGS: the NaN test is one compare of the sort's rank-0 output, which
  // every NaN among the 128 keys reaches (the NaN-propagating mins of its
  // cone, gen_networks.py NAN_CONE_TAGS) -- where a packed-FMA chain over the
  // loads took 34 instructions per wave
  sort_full<kHalf>(x);
  // NP == 1: the waves swap their rank-0 outputs instead of flags -- B's is
  // row 0 of the parity wave 1 hands over anyway, A's goes through the
  // partial-sum slot (free until barrier 3) -- and both test the same pair
  // per lane with one compare whose mask the compiler knows is uniform
  // (llvm.amdgcn.fcmp): 1 VALU where the flag round trip took 13.
  constexpr bool kSwap0 = FLAGS && NP == 1;
  uint64_t nan = 0;
  if constexpr (FLAGS && !kSwap0) nan = unordered_mask(bits_f(x[0]), bits_f(x[0]));
  const bool has_nan = FLAGS && !kSwap0 && uniform(nan != 0);
  pin(x);
  // Batcher's odd-even merge of A (wave 0) and B (wave 1), split by parity:
  // v = merge(A_even, B_even) in wave 0, w = merge(A_odd, B_odd) in wave 1,
  // and the merged order is c_0 = v_0, c_{2i-1} = min(v_i, w_{i-1}),
  // c_{2i} = max(v_i, w_{i-1}).  Each wave hands the parity it does not merge
  // to the other (64 keys, 16 KB): wave 0 A_odd through R0, wave 1 B_even
  // through R1.
  // (the distinct asm after each side's stores keeps LLVM from sinking both
  // into one store sequence fed by moves or selects)
  W32 r0 = reinterpret_cast<W32>(im), r1 = r0 + kHalf / 2 * 64;
  auto part = (float __attribute__((address_space(3)))*)(im + kHalf / 4 * 64);
  if (h == 0) {
#pragma unroll
    for (int j = 0; j < kHalf / 2; ++j) r0[j * 64 + lane] = raw(x[2 * j + 1]);
    if constexpr (kSwap0) part[lane] = bits_f(x[0]);
    asm volatile("; parity hand-off, wave 0" ::: "memory");
  } else {
#pragma unroll
    for (int j = 0; j < kHalf / 2; ++j) r1[j * 64 + lane] = raw(x[2 * j]);
    asm volatile("; parity hand-off, wave 1" ::: "memory");
  }
  if constexpr (FLAGS && !kSwap0) {
    if (lane == 0) flags[2 * pr + h] = has_nan ? 1 : 0;
  }
  block_sync();  // 1: both parities in the image
  // kSwap0: A's rank-0 output (its slot) against B's (row 0 of R1), the same
  // pair per lane in both waves.  A block holding a NaN finishes the float
  // path on garbage and the caller re-runs it on the keys (*redo): a call
  // here, with the sorted halves live on the other path, made LLVM spill ~20
  // of them around it, and one at each return kept wave 0's sums live across
  // wave 1's.  Every image read of the float path has completed at barrier
  // 3, before pair_keys writes.
  if constexpr (kSwap0)
    *redo = __builtin_amdgcn_fcmpf(part[lane], __uint_as_float(row_at(r1, 0, lane)), 8 /* unordered */) != 0;
  if constexpr (FLAGS && !kSwap0) {  // block-wide (same barriers for every pair)
    if (uniform((flags[0] | flags[1] | (NP > 1 ? flags[2] | flags[3] : 0) | (NP > 2 ? flags[4] | flags[5] : 0)) != 0))
      return pair_keys<RULE, PAD>(P, c0, lane_off, im, h, lane, K, pd.lo, pd.m);
  }
  {
    constexpr int b = (2 * kHalf * 2) / 10;  // 51: ranks b..2*kHalf-b-1 = 51..204 kept
    constexpr int Q = kHalf / 2;             // 64
    constexpr int I0 = (b + 1) / 2;          // 26: c_51 = min(v_26, w_25)
    constexpr int IM = kHalf / 2;            // 64: c_127 = min(v_64, w_63), c_128 = max(...)
    constexpr int I1 = kHalf - I0;           // 102: c_204 = max(v_102, w_101)
    constexpr int NX = IM - I0 + 1;          // 39 values cross per wave
    // wave 0 sends v_26..v_64 through R1, wave 1 w_63..w_101 through R0 --
    // each rewrites only the region it read (constant indices: a runtime
    // offset into m would put m in scratch)
    T m[kHalf];
    if (h == 0) {  // v = merge(A_even, B_even): ranks I0..I1 of it
#pragma unroll
      for (int j = 0; j < Q; ++j) {
        m[j] = x[2 * j];
        m[Q + j] = from_raw<T>(row_at(r1, j, lane));
      }
      net_merge128_r26_102<true>(m);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      send_run<I0, NX>(r1, m, lane);
    } else {       // w = merge(A_odd, B_odd): ranks I0-1..I1-1
#pragma unroll
      for (int j = 0; j < Q; ++j) {
        m[j] = from_raw<T>(row_at(r0, j, lane));
        m[Q + j] = x[2 * j + 1];
      }
      net_merge128_r25_101<true>(m);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      send_run<IM - 1, NX>(r0, m, lane);
    }
    block_sync();  // 2: the crossing values in the image
    if (h == 1) {  // c_51..c_127, ascending sum from +0
      T c[2 * (IM - I0) + 1];
#pragma unroll
      for (int i = I0; i < IM; ++i) {
        const T vi = from_raw<T>(row_at(r1, i - I0, lane));
        c[2 * (i - I0)] = min(vi, m[i - 1]);
        c[2 * (i - I0) + 1] = max(vi, m[i - 1]);
      }
      c[2 * (IM - I0)] = min(from_raw<T>(row_at(r1, IM - I0, lane)), m[IM - 1]);
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 2 * (IM - I0) + 1; ++k) {
        const float s = __fadd_rn(acc, val(c[k]));
        acc = !PAD || k < pd.m ? s : acc;  // PAD: padded rank b + k is kept iff k < m
      }
      part[lane] = acc;
      block_sync();  // 3: the partial sum of ranks 51..127 in its slot
      return acc;  // unused (wave 1 stores nothing): no constant to materialise
    }
    T c[2 * (I1 - IM) + 1];  // c_128..c_204
    c[0] = max(m[IM], from_raw<T>(row_at(r0, 0, lane)));
#pragma unroll
    for (int i = IM + 1; i <= I1; ++i) {
      const T wi = from_raw<T>(row_at(r0, i - IM, lane));  // w_{i-1}
      c[2 * (i - IM) - 1] = min(m[i], wi);
      c[2 * (i - IM)] = max(m[i], wi);
    }
    block_sync();  // 3
    float acc = part[lane];
#pragma unroll
    for (int k = 0; k < 2 * (I1 - IM) + 1; ++k) {
      const float s = __fadd_rn(acc, val(c[k]));
      acc = !PAD || 2 * (IM - I0) + 1 + k < pd.m ? s : acc;  // padded rank b + 77 + k
    }
    if constexpr (PAD) return acc / static_cast<float>(pd.m);
    return div_const<2 * kHalf - 2 * b>(acc);  // = acc / 154.f, bit for bit (robust_nets.h)
  }
}

// This wave's 128 inputs of the tile.  Every load is the saddr form: the
// peer row's base plus the tile start in SGPRs, one 32-bit lane offset shared
// by all 128 loads -- no 64-bit VGPR address per load.  The asm keeps LLVM
// from re-associating the tile start into the lane offset.
// PAD: slots >= K read their pad row (KEYS: the key path's), lo of them the
// bottom one.
template <bool PAD = false, bool KEYS = false>
__device__ __forceinline__ void load_half(uint32_t (&v)[kHalf], const float* const* P, int64_t c0,
                                          uint32_t lane_off, int h, int K = 2 * kHalf, int lo = 0) {
  const uint64_t prow = reinterpret_cast<uint64_t>(pad_row(KEYS, false));  // the top row follows it
#pragma unroll
  for (int j = 0; j < kHalf; ++j) {
    const int slot = h * kHalf + j;
    uint64_t row = reinterpret_cast<uint64_t>(table_at(P, PAD ? min(slot, K - 1) : slot) + c0);
    if (PAD && slot >= K) row = prow + (slot - K >= lo ? kPadRowBytes : 0u);
    asm("" : "+s"(row));
    const P2P_GLOBAL float* src =
        reinterpret_cast<const P2P_GLOBAL float*>(reinterpret_cast<const P2P_GLOBAL char*>(row) + lane_off);
    // PAD: through the caches (every wave of the chip reads the same pad
    // rows: streamed, they would all go to one L2 channel)
    v[j] = __float_as_uint(PAD ? *src : __builtin_nontemporal_load(src));
  }
  __builtin_amdgcn_sched_barrier(0);  // all loads in flight before the first use
}

// The uint32-key network for a block holding a NaN.  Out of line and
// re-loading its inputs, so the float path's 128 values are not also held
// live for this one (inlined, the two paths took 320-390 VGPRs).
template <int RULE, bool PAD>
__device__ __attribute__((noinline)) float pair_keys(const float* const* P, int64_t c0, uint32_t lane_off, Img im,
                                                     int h, int lane, int K, int lo, int m) {
  // arguments arrive in VGPRs: make the wave-uniform ones scalar again
  P = reinterpret_cast<const float* const*>(uniform_u64(reinterpret_cast<uint64_t>(P)));
  c0 = static_cast<int64_t>(uniform_u64(static_cast<uint64_t>(c0)));
  h = __builtin_amdgcn_readfirstlane(h);
  Pads pd;
  pd.lo = __builtin_amdgcn_readfirstlane(lo);
  pd.m = __builtin_amdgcn_readfirstlane(m);
  K = __builtin_amdgcn_readfirstlane(K);
  uint32_t v[kHalf];
  load_half<PAD, true>(v, P, c0, lane_off, h, K, pd.lo);
  if constexpr (RULE == P2P_RULE_MEDIAN)
    return median_pair<uint32_t, false, PAD>(v, im, h, lane, nullptr, P, c0, lane_off, K, pd);
  else return pair_body<RULE, kx, false, PAD>(v, im, h, lane, nullptr, P, c0, lane_off, K, pd);  // kx: max as a ^ b ^ min
}

// One 64-coordinate tile of the pair kernels.  SMALL (flat buffers of at
// most kNarrowMaxN floats): the tile start rides in the 32-bit lane offset and each peer
// row's pointer is the scalar base as loaded -- no 64-bit scalar add per load
// (256 SALU instructions per wave and tile).
// NP wave pairs per block: pair pr takes coordinates 64 pr .. 64 pr + 63 of
// the block's tile (its own LDS image, im already offset).
template <int RULE, bool SEGS, bool SMALL, bool PAD, int NP = 1>
__device__ __forceinline__ void pair_tile(const float* const* __restrict__ peers, const Seg* __restrict__ segs,
                                          int nseg, int64_t n, float* w, float* out, float lr, Img im,
                                          int __attribute__((address_space(3)))* flags, int64_t t, int K, int trim_b) {
  const int h = __builtin_amdgcn_readfirstlane(static_cast<int>(NP == 1 ? tid_x() >> 6 : (tid_x() >> 6) & 1));
  const int pr = NP == 1 ? 0 : __builtin_amdgcn_readfirstlane(static_cast<int>(tid_x() >> 7));
  const int lane = tid_x() & 63;
  const float* const* P = peers;
  float* W = w;
  float* O = out;
  int64_t N = n, c0 = t * (kPairTile * NP) + pr * kPairTile;
  if constexpr (SEGS) {
    const Seg s = load_segment(segs, nseg, t);
    P = s.peers;
    W = s.w;
    O = s.out;
    N = s.n;
    c0 = (t - s.tile_begin) * (kPairTile * NP) + pr * kPairTile;
  }
  // Dead lanes of a ragged tail re-read the last element; with NP > 1 a
  // whole wave pair can lie past the end (it still joins the block's
  // barriers), so its row base is clamped too: 0 <= lane_off < 256 whenever
  // the base carries the tile start.
  // row base offset (SMALL: 0, the whole offset rides per lane; never for
  // PAD, whose pad rows are one tile wide)
  // NARROW (SMALL flat buffers, n <= kNarrowMaxN): every index a 32-bit byte
  // offset -- one add and one v_min_u32 per lane, and w / out are read and
  // written through buffer descriptors at that same offset (no 64-bit
  // address); the 64-bit form costs ~9 VALU more per wave.
  constexpr bool NARROW = SMALL && !PAD && !SEGS;
  const int64_t i = c0 + lane;
  const int64_t cb = SMALL && !PAD ? 0 : (c0 < N ? c0 : N - 1);
  uint32_t lane_off;
  bool live;
  if constexpr (NARROW) {
    const uint32_t at = static_cast<uint32_t>(c0) * 4u + lane * 4u, last = static_cast<uint32_t>(N - 1) * 4u;
    live = at <= last;
    lane_off = min(at, last);
  } else {
    live = i < N;
    lane_off = static_cast<uint32_t>((live ? i : N - 1) - cb) * 4u;
  }
  Pads pd;
  if constexpr (PAD) {
    pd.lo = RULE == P2P_RULE_MEDIAN ? (2 * kHalf - 1) / 2 - (K - 1) / 2 : (2 * kHalf * 2) / 10 - trim_b;
    pd.m = K - 2 * trim_b;
  }
  uint32_t v[kHalf];
  load_half<PAD>(v, P, cb, lane_off, h, K, pd.lo);
  // One domain per block: the float network unless either half holds a NaN
  // (flags swapped at the first barrier, no barrier of their own).
  float agg;
  if constexpr (RULE == P2P_RULE_MEDIAN)
    agg = median_pair<fk, true, PAD, NP>(v, im, h, lane, flags, P, cb, lane_off, K, pd, pr);
  else {
    bool redo = false;  // NP == 1: the NaN test's outcome, acted on here (pair_body)
    agg = pair_body<RULE, fk, true, PAD, NP>(v, im, h, lane, flags, P, cb, lane_off, K, pd, pr, &redo);
    if (NP == 1 && redo) agg = pair_keys<RULE, PAD>(P, cb, lane_off, im, h, lane, K, pd.lo, pd.m);
  }
  if (h == 0 && live) {  // wave 0 holds the aggregate
    if constexpr (NARROW) {  // a live lane's offset is its coordinate's
      constexpr int kSt = P2P_ROBUST_STORE_AUX < 0 ? 0 : P2P_ROBUST_STORE_AUX;
      if (O) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(agg), flat_rsrc(O), lane_off, 0, kSt);
      if (W) {
        const auto r = flat_rsrc(W);
        const float wv = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, lane_off, 0, 0));
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(apply_lr(wv, lr, agg)), r, lane_off, 0, kSt);
      }
    } else {
      if (O) stg(O + i, agg);
      if (W) stg(W + i, apply_lr(ldg(W + i), lr, agg));
    }
  }
}

// Trimmed mean: two 16 KB parity regions + the partial sums (256 B), 2 waves
// per SIMD.
template <bool SEGS, bool SMALL = false, bool PAD = false>
__global__ __launch_bounds__(128 * kTrimPairs) __attribute__((amdgpu_waves_per_eu(2))) void robust_pair_kernel(
    const float* const* __restrict__ peers, const Seg* __restrict__ segs, int nseg, int64_t n, float* w,
    float* out, float lr, int64_t ntiles, unsigned gx, int K, int trim_b) {
  constexpr int kImg = kHalf / 4 * 64 + 16;
  __shared__ u32x4 img_raw[kImg * kTrimPairs];
  __shared__ int nan_flag[2 * kTrimPairs];
  const int64_t t = tile_id(gx);
  // block-uniform; SMALL: fewer than 2^24 tiles, a 32-bit scalar compare
  if (SMALL ? static_cast<uint32_t>(t) >= static_cast<uint32_t>(ntiles) : t >= ntiles) return;
  const int pr = kTrimPairs == 1 ? 0 : __builtin_amdgcn_readfirstlane(static_cast<int>(tid_x() >> 7));
  pair_tile<P2P_RULE_TRIMMED, SEGS, SMALL, PAD, kTrimPairs>(peers, segs, nseg, n, w, out, lr, (Img)img_raw + pr * kImg,
                                                (int __attribute__((address_space(3)))*)nan_flag, t, K, trim_b);
}

// Median: per wave pair a 16 KB image (B's kept half) + both max(lo)
// (512 B); kMedianPairs pairs per block, 3 waves per SIMD (<= 168 VGPRs).
template <bool SEGS, bool SMALL = false, bool PAD = false>
__global__ __launch_bounds__(128 * kMedianPairs) __attribute__((amdgpu_waves_per_eu(3))) void
robust_median_pair_kernel(const float* const* __restrict__ peers, const Seg* __restrict__ segs, int nseg, int64_t n,
                          float* w, float* out, float lr, int64_t ntiles, unsigned gx, int K, int trim_b) {
  constexpr int kImg = kHalf / 8 * 64 + 32;
  __shared__ u32x4 img_raw[kImg * kMedianPairs];
  __shared__ int nan_flag[2 * kMedianPairs];
  const int64_t t = tile_id(gx);
  if (SMALL ? static_cast<uint32_t>(t) >= static_cast<uint32_t>(ntiles) : t >= ntiles) return;  // block-uniform
  const int pr = kMedianPairs == 1 ? 0 : __builtin_amdgcn_readfirstlane(static_cast<int>(tid_x() >> 7));
  pair_tile<P2P_RULE_MEDIAN, SEGS, SMALL, PAD, kMedianPairs>(peers, segs, nseg, n, w, out, lr,
                                                             (Img)img_raw + pr * kImg,
                                                             (int __attribute__((address_space(3)))*)nan_flag, t,
                                                             K, trim_b);
}

}  // namespace p2p

using namespace p2p;

// Coordinates per block tile of the pair kernels.
extern "C" P2P_INTERNAL int64_t p2p_robust_pair_tile(int32_t rule) {
  return kPairTile * (rule == P2P_RULE_MEDIAN ? kMedianPairs : kTrimPairs);
}

// Whether the pair kernels take (rule, K, b): K = 256 with the median or
// b = 51 as built; K in 129..255 (or another b) padded to 256 when the pads
// fit (the median always; the trimmed mean while b <= 51, K - b <= 205 and
// K - 2b <= 154, which every K in 129..256 meets at the default 0.2 trim).
extern "C" P2P_INTERNAL int32_t p2p_robust_pair_fits(int32_t rule, int32_t k, int32_t trim_b) {
  if (k <= kHalf || k > 2 * kHalf) return 0;
  if (rule == P2P_RULE_MEDIAN) return 1;
  return trim_b >= 0 && trim_b <= 51 && k - trim_b <= 205 && k - 2 * trim_b >= 1 && k - 2 * trim_b <= 154;
}

// K in 129..256 (p2p_robust_pair_fits): one block per 64-coordinate tile
// (flat: ceil(n / 64); segment table: `tiles`, tile_begin in units of 64), on
// a 2-D grid beyond 2^24 tiles.  The unpadded kernels for K = 256 with the
// median or b = 51, the PAD kernels otherwise.
extern "C" P2P_INTERNAL void p2p_robust_pair_launch(const float* const* peers, const p2p_segment_t* segs,
                                                    int32_t nseg, int64_t tiles, int32_t rule, int32_t k,
                                                    int32_t trim_b, int64_t n, float* w, float* out, float lr,
                                                    p2p_stream_t stream) {
  const hipStream_t st = static_cast<hipStream_t>(stream);
  const int np = rule == P2P_RULE_MEDIAN ? kMedianPairs : kTrimPairs;  // p2p_robust_pair_tile
  const int64_t ntiles = segs ? tiles : ceil_div(n, kPairTile * np);
  const TileGrid tg = tile_grid(ntiles, 128 * np);  // 2 x 64 lanes per 64 coordinates: 1-D, n > 2^31 would wrap
  if (tg.gx == 0) return;
  const dim3 g(tg.gx, tg.gy), b(2 * 64 * np);
  const bool pad = !(k == 2 * kHalf && (rule == P2P_RULE_MEDIAN || trim_b == 51));
  const bool small = !segs && n <= kNarrowMaxN;
#define P2P_PAIR_ARGS g, b, 0, st, peers, segs, nseg, n, w, out, lr, ntiles, tg.gx, k, trim_b
#define P2P_PAIR_LAUNCH(KERNEL)                                                                \
  do {                                                                                         \
    if (pad) {                                                                                 \
      if (segs) hipLaunchKernelGGL((KERNEL<true, false, true>), P2P_PAIR_ARGS);                \
      else hipLaunchKernelGGL((KERNEL<false, false, true>), P2P_PAIR_ARGS);                    \
    } else {                                                                                   \
      if (segs) hipLaunchKernelGGL((KERNEL<true, false, false>), P2P_PAIR_ARGS);               \
      else if (small) hipLaunchKernelGGL((KERNEL<false, true, false>), P2P_PAIR_ARGS);         \
      else hipLaunchKernelGGL((KERNEL<false, false, false>), P2P_PAIR_ARGS);                   \
    }                                                                                          \
  } while (0)
  if (rule == P2P_RULE_MEDIAN) P2P_PAIR_LAUNCH(robust_median_pair_kernel);
  else P2P_PAIR_LAUNCH(robust_pair_kernel);
#undef P2P_PAIR_LAUNCH
#undef P2P_PAIR_ARGS
}
