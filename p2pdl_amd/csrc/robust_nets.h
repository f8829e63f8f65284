// Register-resident comparator networks over uint32 total-order keys
// (generated into networks.inc by gen_networks.py), shared by robust.hip
// (one lane / wave group per coordinate) and robust_lds.hip (L lanes per
// coordinate, LDS-DMA staged).
#pragma once
#include "p2p_common.h"

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

// Any NaN among the n values of any lane of the wave (wave-uniform).
template <int N>
__device__ __forceinline__ bool wave_has_nan(const uint32_t (&bits)[N]) {
  static_assert(N % 2 == 0, "pairs");
  uint64_t m = 0;
#pragma unroll
  for (int j = 0; j < N / 2; ++j) m |= unordered_mask(__uint_as_float(bits[j]), __uint_as_float(bits[j + N / 2]));
  return m != 0;
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
#define P2P_CE(a, b) ce<ASC>((a), (b))
#define P2P_MIN(a, b) (a) = (ASC ? min((a), (b)) : max((a), (b)))
#define P2P_MAX(a, b) (b) = (ASC ? max((a), (b)) : min((a), (b)))
#include "networks.inc"
#undef P2P_CE
#undef P2P_MIN
#undef P2P_MAX

template <int KP, bool ASC = true, typename T> __device__ __forceinline__ void sort_full(T (&v)[KP]) {
  if constexpr (KP == 2) net_sort2<ASC>(v);
  else if constexpr (KP == 4) net_sort4<ASC>(v);
  else if constexpr (KP == 8) net_sort8<ASC>(v);
  else if constexpr (KP == 16) net_sort16<ASC>(v);
  else if constexpr (KP == 32) net_sort32<ASC>(v);
  else if constexpr (KP == 64) net_sort64<ASC>(v);
  else net_sort128<ASC>(v);
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
template <int KP, int MODE, typename T> __device__ __forceinline__ void run_special(T (&v)[KP]) {
  if constexpr (KP == 64 && MODE == 1) net_median64<true>(v);
  else if constexpr (KP == 128 && MODE == 1) net_median128<true>(v);
  else if constexpr (KP == 64 && MODE == 2) net_trim64_b12<true>(v);
  else net_trim128_b25<true>(v);
}

}  // namespace p2p
