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
// Branch-free (arithmetic shift masks): 3 VALU ops, no VCC hazard s_nops.
__device__ __forceinline__ uint32_t f2key(uint32_t b) {
  return b ^ (static_cast<uint32_t>(static_cast<int32_t>(b) >> 31) | 0x80000000u);
}
__device__ __forceinline__ uint32_t key2f(uint32_t k) {
  return k ^ (~static_cast<uint32_t>(static_cast<int32_t>(k) >> 31) | 0x80000000u);
}

// w + lr*agg with the multiply and the add each rounded (no FMA), matching
// reference aggregator/aggregation.py:38 (`w += 0.1 * acc` on CPU).
__device__ __forceinline__ float apply_lr(float w, float lr, float agg) {
  return __fadd_rn(w, __fmul_rn(lr, agg));
}

// Loads through the GLOBAL address space.  A generic pointer makes hipcc emit
// flat_load, which also counts on lgkmcnt: every s_waitcnt lgkmcnt(0) for the
// next scalar (pointer-table) load then drains all outstanding data loads.
#define P2P_GLOBAL __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ T ldg_nt(const T* p) {
  return __builtin_nontemporal_load((const P2P_GLOBAL T*)(p));
}
template <typename T>
__device__ __forceinline__ T ldg(const T* p) {
  return *(const P2P_GLOBAL T*)(p);
}
template <typename T>
__device__ __forceinline__ void stg(T* p, T v) {
  *(P2P_GLOBAL T*)(p) = v;
}

// Entry k of a device pointer table, read through the CONSTANT address space
// so a wave-uniform index becomes one scalar s_load (the table is read-only).
#define P2P_CONST __attribute__((address_space(4)))
template <typename T>
__device__ __forceinline__ T* table_at(T* const* table, int k) {
  return reinterpret_cast<T*>(((const P2P_CONST uint64_t*)(table))[k]);
}
// A wave-uniform field of a host-built, launch-read-only table (tile lists,
// chunk lists, segment descriptors) as a scalar s_load.  Read through GLOBAL
// (ldg) it is a vector load + readfirstlane, and hipcc waits for it with
// s_waitcnt vmcnt(0): in a loader wave that drains the whole LDS-DMA ring,
// in a consumer wave it waits out the previous tile's stores.
template <typename T>
__device__ __forceinline__ T ldc(const T* p) {
  return *(const P2P_CONST T*)(p);
}

// Work-item / work-group ids as intrinsics (the grid size is a kernel
// argument where a loop strides by it).  The robust
// kernels are built with -mno-amdgpu-ieee, which keeps the device library's
// threadIdx / blockIdx helpers (__ockl_get_*, built IEEE) from
// inlining: each became a call returning a VGPR, so block-uniform values --
// tile bases, peer row addresses -- were computed per lane as if divergent.
__device__ __forceinline__ uint32_t tid_x() { return __builtin_amdgcn_workitem_id_x(); }
__device__ __forceinline__ uint32_t bid_x() { return __builtin_amdgcn_workgroup_id_x(); }

__device__ __forceinline__ uint64_t uniform_u64(uint64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(x));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(x >> 32));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// The descriptor of the segment owning tile `t` (segments sorted by
// tile_begin), read through the scalar path: every field is forced
// wave-uniform so the peer table and base pointers live in SGPRs and the
// per-peer pointer loads are s_load, not per-lane vector loads.
__device__ __forceinline__ Seg load_segment(const Seg* segs, int nseg, int64_t t) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    const int64_t tb = ldc(&segs[mid].tile_begin);
    if (tb <= t) lo = mid; else hi = mid - 1;
    lo = __builtin_amdgcn_readfirstlane(lo);
    hi = __builtin_amdgcn_readfirstlane(hi);
  }
  const Seg* sp = segs + lo;
  Seg s;
  s.peers = ldc(&sp->peers);
  s.w = ldc(&sp->w);
  s.out = ldc(&sp->out);
  s.n = ldc(&sp->n);
  s.tile_begin = ldc(&sp->tile_begin);
  return s;
}

// Wave-uniform: are all peer pointers (and w/out) 16-B aligned?
__device__ __forceinline__ bool all_aligned16(const float* const* peers, int K, const float* w,
                                              const float* out) {
  uintptr_t m = reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(out);
  for (int k = 0; k < K; ++k) m |= reinterpret_cast<uintptr_t>(table_at(peers, k));
  return (m & 15) == 0;
}

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// One block per tile over a 2-D grid.  An AQL dispatch counts work-items in
// 32 bits per dimension: one 128-lane block per 64 or 128 coordinates in x
// alone would wrap past 2^31 / 2^32 coordinates and leave the rest of the
// buffer untouched.  Tile t = blockIdx.y * gx + blockIdx.x with gx <= 2^24
// blocks of 128 lanes (2^31 work-items per row; fewer blocks for larger
// ones); the surplus blocks of the last row exit at once.
constexpr int64_t kMaxGridX = int64_t(1) << 24;
struct TileGrid {
  unsigned gx, gy;
};
__host__ inline TileGrid tile_grid(int64_t tiles, int block = 128) {
  const int64_t cap = block <= 128 ? kMaxGridX : (int64_t(1) << 31) / block;
  const int64_t gx = tiles < cap ? tiles : cap;
  return TileGrid{static_cast<unsigned>(gx), static_cast<unsigned>(gx > 0 ? ceil_div(tiles, gx) : 0)};
}
__device__ __forceinline__ int64_t tile_id(unsigned gx) {
  return static_cast<int64_t>(__builtin_amdgcn_workgroup_id_y()) * gx + __builtin_amdgcn_workgroup_id_x();
}

}  // namespace p2p
