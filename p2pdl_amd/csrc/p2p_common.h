// Shared definitions for the gfx950 kernels behind include/p2pdl.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/p2pdl.h"

#define P2P_INTERNAL __attribute__((visibility("hidden")))

namespace p2p {

constexpr int kBlock = 256;  // 4 waves of 64 lanes

// Per-segment descriptor for a state_dict of L tensors (device-resident).
// Layout must match p2p_segment_t in include/p2pdl.h.
using Seg = p2p_segment_t;

// IEEE total order on float bits mapped to an unsigned key:
// -NaN < -inf < ... < -0 < +0 < ... < +inf < +NaN.
__device__ __forceinline__ uint32_t f2key(uint32_t b) {
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ uint32_t key2f(uint32_t k) {
  return (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
}

// w + lr*agg with the multiply and the add each rounded (no FMA), matching
// reference aggregator/aggregation.py:38 (`w += 0.1 * acc` on CPU).
__device__ __forceinline__ float apply_lr(float w, float lr, float agg) {
  return __fadd_rn(w, __fmul_rn(lr, agg));
}

// Binary search of the segment owning tile `t` (segments sorted by tile_begin).
__device__ __forceinline__ int find_segment(const Seg* segs, int nseg, int64_t t) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (segs[mid].tile_begin <= t) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace p2p
