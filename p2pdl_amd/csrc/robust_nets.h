// Register-resident comparator networks over uint32 total-order keys
// (generated into networks.inc by gen_networks.py), shared by robust.hip
// (one lane / wave group per coordinate) and robust_lds.hip (L lanes per
// coordinate, LDS-DMA staged).
#pragma once
#include "p2p_common.h"

namespace p2p {

template <bool ASC, typename T>
__device__ __forceinline__ void ce(T& a, T& b) {
  const T lo = min(a, b), hi = max(a, b);
  if constexpr (ASC) { a = lo; b = hi; } else { a = hi; b = lo; }
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
  else net_bmerge64<true>(v);
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
