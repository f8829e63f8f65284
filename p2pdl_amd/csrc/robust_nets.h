// Register-resident comparator networks over uint32 total-order keys
// (generated into networks.inc by gen_networks.py), shared by robust.hip
// (one lane / wave group per coordinate) and robust_lds.hip (L lanes per
// coordinate, LDS-DMA staged).
#pragma once
#include "p2p_common.h"

namespace p2p {

template <bool ASC>
__device__ __forceinline__ void ce(uint32_t& a, uint32_t& b) {
  const uint32_t lo = min(a, b), hi = max(a, b);
  if constexpr (ASC) { a = lo; b = hi; } else { a = hi; b = lo; }
}
#define P2P_CE(a, b) ce<ASC>((a), (b))
#define P2P_MIN(a, b) (a) = (ASC ? min((a), (b)) : max((a), (b)))
#define P2P_MAX(a, b) (b) = (ASC ? max((a), (b)) : min((a), (b)))
#include "networks.inc"
#undef P2P_CE
#undef P2P_MIN
#undef P2P_MAX

template <int KP, bool ASC = true> __device__ __forceinline__ void sort_full(uint32_t (&v)[KP]);
#define P2P_SORT(KP) \
  template <> __device__ __forceinline__ void sort_full<KP, true>(uint32_t (&v)[KP]) { net_sort##KP<true>(v); } \
  template <> __device__ __forceinline__ void sort_full<KP, false>(uint32_t (&v)[KP]) { net_sort##KP<false>(v); }
P2P_SORT(2) P2P_SORT(4) P2P_SORT(8) P2P_SORT(16) P2P_SORT(32) P2P_SORT(64) P2P_SORT(128)
#undef P2P_SORT

// Sorts a bitonic sequence of KP keys ascending (half-cleaners n/2 .. 1).
template <int KP> __device__ __forceinline__ void bmerge(uint32_t (&v)[KP]);
template <> __device__ __forceinline__ void bmerge<32>(uint32_t (&v)[32]) { net_bmerge32<true>(v); }
template <> __device__ __forceinline__ void bmerge<64>(uint32_t (&v)[64]) { net_bmerge64<true>(v); }

// MODE 0: generic (full sort + runtime rank / trim);
// MODE 1: pruned median network for K == KP;
// MODE 2: pruned trimmed network for K == KP, b == floor(0.2 KP).
template <int KP, int MODE> __device__ __forceinline__ void run_special(uint32_t (&v)[KP]);
template <> __device__ __forceinline__ void run_special<64, 1>(uint32_t (&v)[64]) { net_median64<true>(v); }
template <> __device__ __forceinline__ void run_special<128, 1>(uint32_t (&v)[128]) { net_median128<true>(v); }
template <> __device__ __forceinline__ void run_special<64, 2>(uint32_t (&v)[64]) { net_trim64_b12<true>(v); }
template <> __device__ __forceinline__ void run_special<128, 2>(uint32_t (&v)[128]) { net_trim128_b25<true>(v); }

}  // namespace p2p
