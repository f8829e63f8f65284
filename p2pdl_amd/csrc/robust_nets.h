// Register-resident comparator networks over uint32 total-order keys
// (generated into networks.inc by gen_networks.py), shared by robust.hip
// (one lane / wave group per coordinate) and robust_lds.hip (L lanes per
// coordinate, LDS-DMA staged).
#pragma once
#include "p2p_common.h"

// The robust kernels' w / out stores: -1 plain (global stores, or buffer
// stores without cache-policy bits); else buffer stores with these bits (bit
// 0 sc0, bit 1 nt, bit 4 sc1) -- the A/B builds' knob (the FedAvg split
// kernel's and the delta's stores won by device-scope sc1).
#ifndef P2P_ROBUST_STORE_AUX
#define P2P_ROBUST_STORE_AUX 18
#endif

namespace p2p {

// NaN-free fast path: the networks run on the float values themselves.
// v_min / v_max / v_med3_f32 order -0 < +0 and keep denormals and +-inf
// exactly as the uint32 total-order keys do (tools/fminmax_probe.hip,
// profiles/r01/probes), so for NaN-free inputs every rank -- and every bit of
// the selected value -- is the same as the key network's, without the key map
// (2 VALU per key in, 2 per key out).  robust.hip / robust_lds.hip are built
// with -mno-amdgpu-ieee -fno-honor-nans, so min / max need no canonicalising
// v_max_f32 x,x per input; the NaN test is therefore an explicit vector
// compare (the compiler would fold isnan away) and a wave with any NaN takes
// the uint32-key network.
struct fk {
  float x;
};
using ::max;  // keep the global (integer / packed) overloads visible next to fk's
using ::min;
__device__ __forceinline__ fk min(fk a, fk b) { return fk{__builtin_fminf(a.x, b.x)}; }
__device__ __forceinline__ fk max(fk a, fk b) { return fk{__builtin_fmaxf(a.x, b.x)}; }

// Lanes of the wave for which a or b is NaN (v_cmp_u_f32 into an SGPR pair).
__device__ __forceinline__ uint64_t unordered_mask(float a, float b) {
  uint64_t m;
  asm volatile("v_cmp_u_f32 %0, %1, %2" : "=s"(m) : "v"(a), "v"(b));
  return m;
}

// a / D correctly rounded (round to nearest even, what `a / float(D)` gives
// under -fhip-fp32-correctly-rounded-divide-sqrt) in five instructions where
// the compiler's IEEE division issues eleven: q0 = a * y with y = RN(1/D),
// the exact residual r = a - q0 * D (one FMA), q1 = q0 + r * y (Markstein's
// correction: correctly rounded when y is within half an ulp of 1/D, q0
// within one ulp of a/D and the quotient normal), and v_div_fixup_f32 for
// the operands the correction cannot take (+-inf: r = inf - inf; NaN).  A
// subnormal quotient rounds onto the fixed 2^-149 grid, where the
// correction misses exact and near ties (108,942 of the 2^32 inputs for D =
// 154, all |a| < 2^-125; below 2^-124 for 40): a wave with a lane below 2^-118 takes the IEEE division
// (one compare and a uniform branch).  tools/div_probe.hip checks the whole
// function against the double quotient for all 2^32 inputs of each divisor.
template <int D>
__device__ __forceinline__ float div_const_fast(float a) {
  constexpr float y = 1.0f / D;
  const float q0 = __fmul_rn(a, y);
  const float r = __builtin_fmaf(-q0, static_cast<float>(D), a);
  return __builtin_amdgcn_div_fixupf(__builtin_fmaf(r, y, q0), static_cast<float>(D), a);
}
template <int D>
__device__ __forceinline__ float div_const(float a) {
  static_assert(D > 0 && D < (1 << 8), "the 2^-118 bound keeps a / D normal for D < 2^8");
  if (__builtin_amdgcn_fcmpf(__builtin_fabsf(a), 0x1p-118f, 4 /* ordered less than */) != 0)
    return a / static_cast<float>(D);
  return div_const_fast<D>(a);
}

// Lanes for which any of the N values at(0) .. at(N-1) is NaN.  NaN
// propagates through v_pk_fma_f32 (a * b + c on float pairs), so each
// instruction folds four more values into a running pair: the first takes
// six, the rest four, and one v_cmp_u_f32 tests the final pair -- about N/4 + 1
// instructions where one compare per two values takes N/2 (the loaded
// values already sit in register pairs: no moves).  An overflowing product,
// inf * 0 or inf - inf also ends in NaN: a false alarm only sends the tile
// to the exact uint32-key network.  Fewer than six values: compares.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v pk_fma(f2v a, f2v b, f2v c) {
  f2v d;
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
// v_maximum3_f32 (IEEE 754-2019 maximum, gfx950): NaN in, NaN out, and no
// NaN from infinities.
__device__ __forceinline__ float maximum3(float a, float b, float c) {
  float d;
  asm volatile("v_maximum3_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
// v_minimum3_f32 likewise (IEEE 754-2019 minimum); not volatile: the
// scheduler may move it like the min it stands for.
__device__ __forceinline__ float minimum3_nv(float a, float b, float c) {
  float d;
  asm("v_minimum3_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ float maximum3_nv(float a, float b, float c) {
  float d;
  asm("v_maximum3_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
// INF_SAFE: the test of a padded network's slots, whose +-inf pad rows meet
// (inf - inf in the FMA chain would send every tile to the key path): two
// v_maximum3 chains, two values per instruction.
template <int N, bool INF_SAFE = false, typename F>
__device__ __forceinline__ uint64_t nan_lanes(F&& at) {
  static_assert(N % 2 == 0, "pairs");
  if constexpr (INF_SAFE && N >= 6) {
    float a = maximum3(at(0), at(1), at(2)), b = maximum3(at(3), at(4), at(5));
    int j = 6;
#pragma unroll
    for (; j + 3 < N; j += 4) {
      a = maximum3(a, at(j), at(j + 1));
      b = maximum3(b, at(j + 2), at(j + 3));
    }
    if constexpr ((N - 6) % 4 == 2) a = maximum3(a, at(N - 2), at(N - 1));
    return unordered_mask(a, b);
  } else if constexpr (N < 6) {
    uint64_t m = 0;
#pragma unroll
    for (int j = 0; j < N / 2; ++j) m |= unordered_mask(at(j), at(j + N / 2));
    return m;
  } else {
    f2v acc = pk_fma(f2v{at(0), at(1)}, f2v{at(2), at(3)}, f2v{at(4), at(5)});
#pragma unroll
    for (int j = 6; j + 3 < N; j += 4) acc = pk_fma(f2v{at(j), at(j + 1)}, f2v{at(j + 2), at(j + 3)}, acc);
    if constexpr ((N - 6) % 4 == 2) acc = pk_fma(f2v{at(N - 2), at(N - 1)}, f2v{1.f, 1.f}, acc);
    return unordered_mask(acc.x, acc.y);
  }
}

// Any NaN among the n values of any lane of the wave (wave-uniform).
template <int N>
__device__ __forceinline__ bool wave_has_nan(const uint32_t (&bits)[N]) {
  return nan_lanes<N>([&](int j) { return __uint_as_float(bits[j]); }) != 0;
}

template <bool ASC, typename T>
__device__ __forceinline__ void ce(T& a, T& b) {
  const T lo = min(a, b), hi = max(a, b);
  if constexpr (ASC) { a = lo; b = hi; } else { a = hi; b = lo; }
}

// uint32 keys whose compare-exchange takes the larger key as a ^ b ^ min(a, b)
// (one v_bitop3) instead of v_max.  Not faster per instruction -- both issue
// in the same slot (tools/sort_probe.hip) -- but the register allocator keeps
// fewer values live: the pruned trimmed mean of 128 drops from 183 to 153
// VGPRs, i.e. from 2 to 3 waves per SIMD (cfg4 trimmed -2.9% time).
struct kx {
  uint32_t k;
};
__device__ __forceinline__ kx min(kx a, kx b) { return kx{::min(a.k, b.k)}; }
__device__ __forceinline__ kx max(kx a, kx b) { return kx{::max(a.k, b.k)}; }
template <bool ASC>
__device__ __forceinline__ void ce(kx& a, kx& b) {
  const uint32_t lo = ::min(a.k, b.k), hi = __builtin_amdgcn_bitop3_b32(a.k, b.k, lo, 0x96);
  if constexpr (ASC) { a.k = lo; b.k = hi; } else { a.k = hi; b.k = lo; }
}
// The same for NaN-free floats: v_min_f32 returns one of its inputs bit for
// bit (-0 < +0), so the larger is again a ^ b ^ min(a, b).
struct fx {
  float x;
};
__device__ __forceinline__ fx min(fx a, fx b) { return fx{__builtin_fminf(a.x, b.x)}; }
__device__ __forceinline__ fx max(fx a, fx b) { return fx{__builtin_fmaxf(a.x, b.x)}; }
template <bool ASC>
__device__ __forceinline__ void ce(fx& a, fx& b) {
  const float lo = __builtin_fminf(a.x, b.x);
  const float hi = __uint_as_float(
      __builtin_amdgcn_bitop3_b32(__float_as_uint(a.x), __float_as_uint(b.x), __float_as_uint(lo), 0x96));
  if constexpr (ASC) { a.x = lo; b.x = hi; } else { a.x = hi; b.x = lo; }
}
// Pad rows of the padded robust kernels (K below the network's size): a pad
// slot loads lane l's word from one of these 256-word rows instead of a peer
// row -- L1/L2-resident, no HBM traffic, no VALU select -- so the network
// sees -inf / +inf (float path) or the bottom / top key (key path: float bits
// 0xFFFFFFFF and 0x7FFFFFFF, which f2key maps to 0 and ~0).
#define P2P_R4(x) x, x, x, x
#define P2P_R16(x) P2P_R4(x), P2P_R4(x), P2P_R4(x), P2P_R4(x)
#define P2P_R128(x) P2P_R16(x), P2P_R16(x), P2P_R16(x), P2P_R16(x), P2P_R16(x), P2P_R16(x), P2P_R16(x), P2P_R16(x)
#define P2P_R256(x) P2P_R128(x), P2P_R128(x)
constexpr unsigned kPadRowBytes = 1024;  // one word per lane of a 256-lane block
__device__ static const uint32_t kPadRows[4][kPadRowBytes / 4] = {
    {P2P_R256(0xFF800000u)}, {P2P_R256(0x7F800000u)}, {P2P_R256(0xFFFFFFFFu)}, {P2P_R256(0x7FFFFFFFu)}};
#undef P2P_R256
#undef P2P_R128
#undef P2P_R16
#undef P2P_R4
// The pad row for (key path?, top of the order?), as a peer row pointer.
__device__ __forceinline__ const float* pad_row(bool keys, bool top) {
  return reinterpret_cast<const float*>(kPadRows[(keys ? 2 : 0) + (top ? 1 : 0)]);
}

// Per-block hook of the generated networks: hook(v, blk) runs before the
// first comparator that reads keys 16*blk .. 16*blk+15 (still the inputs).
struct NoHook {
  template <typename V>
  __device__ __forceinline__ void operator()(V&, int) const {}
};
__device__ __forceinline__ float bits_f(uint32_t k) { return __uint_as_float(k); }
__device__ __forceinline__ float bits_f(fk x) { return x.x; }
__device__ __forceinline__ float bits_f(fx x) { return x.x; }
// The NaN test of the float networks (nan_lanes: packed FMAs), block by
// block as the network first reads it: the test waits only for that
// block's loads (a whole-wave test up front waited for every load before the
// first comparator: median256 -3.5% time without it).
// G blocks per test, blocks from FIRST on; blocks from SAFE on may hold pad
// rows (nan_lanes INF_SAFE).
template <int G = 1, int FIRST = 0, int SAFE = 1 << 20>
struct NanHook {
  uint64_t& m;
  template <typename T, int KP>
  __device__ __forceinline__ void operator()(T (&v)[KP], int blk) const {
    if (blk % G != 0 || blk < FIRST) return;
    constexpr int N = 16 * G < KP ? 16 * G : KP;
    if (blk >= SAFE) m |= nan_lanes<N, true>([&](int j) { return bits_f(v[16 * blk + j]); });
    else m |= nan_lanes<N>([&](int j) { return bits_f(v[16 * blk + j]); });
  }
};
__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
  return max(min(a, b), min(max(a, b), c));  // -> v_med3_u32
}

// The generated networks' instructions (gen_networks.py lowers every
// comparator network to one of these per computed value).  ASC = false is the
// mirror image: min <-> max, med3 unchanged.  Three-input forms become
// v_min3 / v_max3 / v_med3 (f32 for fk / fx, u32 for keys).
template <bool ASC, typename T>
__device__ __forceinline__ T lo2(T a, T b) { return ASC ? min(a, b) : max(a, b); }
template <bool ASC, typename T>
__device__ __forceinline__ T hi2(T a, T b) { return ASC ? max(a, b) : min(a, b); }
// The other output of a comparator whose `lo` is computed too: plain max for
// fk / uint32_t; a ^ b ^ lo (one v_bitop3) for kx / fx, which keeps fewer
// values live (see kx above).
template <bool ASC, typename T>
__device__ __forceinline__ T hi_sib(T a, T b, T) { return hi2<ASC>(a, b); }
template <bool ASC>
__device__ __forceinline__ kx hi_sib(kx a, kx b, kx lo) { return kx{static_cast<uint32_t>(__builtin_amdgcn_bitop3_b32(a.k, b.k, lo.k, 0x96))}; }
template <bool ASC>
__device__ __forceinline__ fx hi_sib(fx a, fx b, fx lo) {
  return fx{__uint_as_float(
      __builtin_amdgcn_bitop3_b32(__float_as_uint(a.x), __float_as_uint(b.x), __float_as_uint(lo.x), 0x96))};
}
template <bool ASC, typename T>
__device__ __forceinline__ T lo3(T a, T b, T c) { return lo2<ASC>(lo2<ASC>(a, b), c); }
template <bool ASC, typename T>
__device__ __forceinline__ T hi3(T a, T b, T c) { return hi2<ASC>(hi2<ASC>(a, b), c); }
// The NaN-propagating mins of a sort's rank-0 cone (gen_networks.py
// NAN_CONE_TAGS): on floats v_minimum3_f32 (v_maximum3 descending) -- NaN in
// any operand gives NaN, otherwise one of the operands bit for bit, -0 < +0,
// exactly what v_min / v_min3 select on NaN-free floats; on keys the plain min.
template <bool ASC, typename T>
__device__ __forceinline__ T lon(T a, T b) { return lo2<ASC>(a, b); }
template <bool ASC, typename T>
__device__ __forceinline__ T lo3n(T a, T b, T c) { return lo3<ASC>(a, b, c); }
template <bool ASC>
__device__ __forceinline__ fk lon(fk a, fk b) { return fk{ASC ? minimum3_nv(a.x, b.x, b.x) : maximum3_nv(a.x, b.x, b.x)}; }
template <bool ASC>
__device__ __forceinline__ fx lon(fx a, fx b) { return fx{ASC ? minimum3_nv(a.x, b.x, b.x) : maximum3_nv(a.x, b.x, b.x)}; }
template <bool ASC>
__device__ __forceinline__ fk lo3n(fk a, fk b, fk c) { return fk{ASC ? minimum3_nv(a.x, b.x, c.x) : maximum3_nv(a.x, b.x, c.x)}; }
template <bool ASC>
__device__ __forceinline__ fx lo3n(fx a, fx b, fx c) { return fx{ASC ? minimum3_nv(a.x, b.x, c.x) : maximum3_nv(a.x, b.x, c.x)}; }
__device__ __forceinline__ uint32_t med3(uint32_t a, uint32_t b, uint32_t c) { return umed3(a, b, c); }
__device__ __forceinline__ kx med3(kx a, kx b, kx c) { return kx{umed3(a.k, b.k, c.k)}; }
__device__ __forceinline__ fk med3(fk a, fk b, fk c) { return fk{__builtin_amdgcn_fmed3f(a.x, b.x, c.x)}; }
__device__ __forceinline__ fx med3(fx a, fx b, fx c) { return fx{__builtin_amdgcn_fmed3f(a.x, b.x, c.x)}; }
#define P2P_LO(a, b) lo2<ASC>((a), (b))
#define P2P_HI(a, b) hi2<ASC>((a), (b))
#define P2P_HIS(a, b, lo) hi_sib<ASC>((a), (b), (lo))
#define P2P_LO3(a, b, c) lo3<ASC>((a), (b), (c))
#define P2P_LON(a, b) lon<ASC>((a), (b))
#define P2P_LO3N(a, b, c) lo3n<ASC>((a), (b), (c))
#define P2P_HI3(a, b, c) hi3<ASC>((a), (b), (c))
#define P2P_MED3(a, b, c) med3((a), (b), (c))
// the round-2 two-input form (gen_networks.py --classic, A/B builds)
#define P2P_CE(a, b) ce<ASC>((a), (b))
#define P2P_MIN(a, b) (a) = (ASC ? min((a), (b)) : max((a), (b)))
#define P2P_MAX(a, b) (b) = (ASC ? max((a), (b)) : min((a), (b)))
#include "networks.inc"
#undef P2P_CE
#undef P2P_MIN
#undef P2P_MAX
#undef P2P_LO
#undef P2P_HI
#undef P2P_HIS
#undef P2P_LO3
#undef P2P_LON
#undef P2P_LO3N
#undef P2P_HI3
#undef P2P_MED3

// keep(a, b, lim): min(a, b) when lim is the bottom of the order, max(a, b)
// when it is the top -- ONE v_med3 against a lane-constant 0 / ~0 (keys) or
// -inf / +inf (floats; v_med3_f32 orders -0 < +0, tools/fminmax_probe.hip).
__device__ __forceinline__ uint32_t keep(uint32_t a, uint32_t p, uint32_t lim) { return umed3(a, p, lim); }
__device__ __forceinline__ fk keep(fk a, fk p, fk lim) { return fk{__builtin_amdgcn_fmed3f(a.x, p.x, lim.x)}; }
__device__ __forceinline__ uint32_t keep_limit(uint32_t, bool hi) { return hi ? 0xFFFFFFFFu : 0u; }
__device__ __forceinline__ fk keep_limit(fk, bool hi) { return fk{hi ? __builtin_inff() : -__builtin_inff()}; }

// a <= b in the total order.  Floats: min(a, b) is a bit for bit (an IEEE
// compare calls -0 and +0 equal, and the two-set search below must not).
__device__ __forceinline__ bool le(uint32_t a, uint32_t b) { return a <= b; }
__device__ __forceinline__ bool le(fk a, fk b) {
  return __float_as_uint(__builtin_fminf(a.x, b.x)) == __float_as_uint(a.x);
}

// max of N values as a tree of v_max3 (ceil((N-1)/2) instructions).
template <int N, typename T>
__device__ __forceinline__ T max_tree(const T* a) {
  if constexpr (N == 1) return a[0];
  else if constexpr (N == 2) return max(a[0], a[1]);
  else if constexpr (N == 3) return max(max(a[0], a[1]), a[2]);
  else {
    constexpr int N1 = N / 3, N2 = (N - N1) / 2, N3 = N - N1 - N2;
    return max(max(max_tree<N1>(a), max_tree<N2>(a + N1)), max_tree<N3>(a + N1 + N2));
  }
}

// ---- median by a two-set search (no merge network) --------------------------
// Lower median of X u Y for X, Y BITONIC of N keys each (rank N-1 of 2N).
// Half-clean both: X_lo = min(X_i, X_{i+N/2}) holds the N/2 smallest of X,
// X_hi the rest, each bitonic again.  If max(X_lo) <= max(Y_lo) (total order)
// every key of X_lo ranks below the wanted one and every key of Y_hi above it,
// so the answer is the lower median of X_hi u Y_lo; else of X_lo u Y_hi.
// Ties choose either branch with the same value.  Per level: N/2 mins and a
// max3 tree per set, one compare, then the kept halves as ONE v_med3 per key
// against a lane-constant limit -- 2.5 VALU per key where a pruned merge
// network pays 2 per comparator over log2 levels.  N = 1: min(X_0, Y_0).
template <int N, typename T>
__device__ __forceinline__ T two_set_median(const T (&x)[N], const T (&y)[N]) {
  if constexpr (N == 1) {
    return min(x[0], y[0]);
  } else {
    constexpr int H = N / 2;
    T xl[H], yl[H];
#pragma unroll
    for (int i = 0; i < H; ++i) {
      xl[i] = min(x[i], x[i + H]);
      yl[i] = min(y[i], y[i + H]);
    }
    const bool d = le(max_tree<H>(xl), max_tree<H>(yl));  // true: keep X_hi, Y_lo
    const T lx = keep_limit(T{}, d), ly = keep_limit(T{}, !d);
    T x2[H], y2[H];
#pragma unroll
    for (int i = 0; i < H; ++i) {
      x2[i] = keep(x[i], x[i + H], lx);
      y2[i] = keep(y[i], y[i + H], ly);
    }
    return two_set_median<H>(x2, y2);
  }
}

// Lower median of four SORTED lists p, q, r, s of N keys (rank 2N-1 of 4N):
// A = p u q and B = r u s split by one flip each, A_lo_j = min(p_j, q_{N-1-j})
// = the N smallest of A (bitonic), A_hi the N largest; the same choice as
// above between A_hi u B_lo and A_lo u B_hi; then two_set_median.  Against
// merging p, q and r, s into sorted halves (two Batcher merges of N + N) and
// the pruned final merge, this drops ~2N log2 N comparators.
template <int N, typename T>
__device__ __forceinline__ T four_list_median(const T (&p)[N], const T (&q)[N], const T (&r)[N], const T (&s)[N]) {
  // max_j min(p_j, q_{N-1-j}) as a v_max3 chain: the N mins are consumed as
  // they are made (a tree would hold 2N more values live next to the lists)
  T ma = min(p[0], q[N - 1]), mb = min(r[0], s[N - 1]);
#pragma unroll
  for (int j = 1; j < N; j += 2) {
    ma = j + 1 < N ? max(max(ma, min(p[j], q[N - 1 - j])), min(p[j + 1], q[N - 2 - j])) : max(ma, min(p[j], q[N - 1 - j]));
    mb = j + 1 < N ? max(max(mb, min(r[j], s[N - 1 - j])), min(r[j + 1], s[N - 2 - j])) : max(mb, min(r[j], s[N - 1 - j]));
  }
  const bool d = le(ma, mb);
  const T lx = keep_limit(T{}, d), ly = keep_limit(T{}, !d);
  T x[N], y[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    x[j] = keep(p[j], q[N - 1 - j], lx);
    y[j] = keep(r[j], s[N - 1 - j], ly);
  }
  return two_set_median<N>(x, y);
}

template <int KP, bool ASC = true, typename T, typename H = NoHook>
__device__ __forceinline__ void sort_full(T (&v)[KP], H&& hook = H{}) {
  if constexpr (KP == 2) net_sort2<ASC>(v);
  else if constexpr (KP == 4) net_sort4<ASC>(v);
  else if constexpr (KP == 8) net_sort8<ASC>(v);
  else if constexpr (KP == 16) net_sort16<ASC>(v, hook);
  else if constexpr (KP == 32) net_sort32<ASC>(v, hook);
  else if constexpr (KP == 64) net_sort64<ASC>(v, hook);
  else net_sort128<ASC>(v, hook);
}

// Sorts a bitonic sequence of KP keys ascending (half-cleaners n/2 .. 1).
template <int KP, typename T> __device__ __forceinline__ void bmerge(T (&v)[KP]) {
  if constexpr (KP == 32) net_bmerge32<true>(v);
  else if constexpr (KP == 64) net_bmerge64<true>(v);
  else net_bmerge128<true>(v);
}

// MODE 0: generic (full sort + runtime rank / trim);
// MODE 1: pruned median network for K == KP;
// MODE 2: pruned trimmed network for K == KP, b == floor(0.2 KP).
template <int KP, int MODE, typename T, typename H = NoHook>
__device__ __forceinline__ void run_special(T (&v)[KP], H&& hook = H{}) {
  if constexpr (KP == 64 && MODE == 1) net_median64<true>(v, hook);
  else if constexpr (KP == 128 && MODE == 1) net_median128<true>(v, hook);
  else if constexpr (KP == 64 && MODE == 2) net_trim64_b12<true>(v, hook);
  else net_trim128_b25<true>(v, hook);
}

}  // namespace p2p
