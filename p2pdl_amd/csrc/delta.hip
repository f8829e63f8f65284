// K4 -- trainer-side local update for gfx950.
//
// Replaces reference node/node.py:273-282 (Node.send_model_to_testers):
//   local_update[key] = current[key] - previous[key]      (:278-279)
//   previous = {key: current[key].clone()}                 (:282)
// and, on the first round (previous is None, :272-275), local_update = current.
// The reference runs one sub kernel and one clone per key (20 B of traffic
// per coordinate over 2L launches); here ONE pass per state_dict reads
// current and previous and writes delta and the new previous: 16 B per
// coordinate, HBM-bound (0.0625 flop/B).  fp32 subtraction is IEEE, so the
// result is bit-exact with torch's CPU/GPU `-`.
//
// Layout: a 256-lane block owns a 1024-float tile, lane l its float4 l ->
// every wave instruction moves one contiguous 1 KiB.  One float4 per lane
// (round 5, tools/delta_lab.hip policy mode, profiles/r05/lab4): 0.767-0.773
// of HBM peak against 0.748-0.758 for four per lane (rounds 1-4), nontemporal
// loads and stores both (each plain variant is 1.5-4% slower), on a box
// whose plain float4 copy reads 0.75-0.78.  Misaligned views and ragged
// tails go element-wise.
#include "p2p_common.h"

namespace p2p {

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kDNV = 1;
constexpr int kDTile = kBlock * 4 * kDNV;  // 1024 floats == P2P_DELTA_TILE
static_assert(kDTile == P2P_DELTA_TILE, "the ABI's delta tile");

__device__ __forceinline__ f4 ld4_nt(const float* p) { return ldg_nt(reinterpret_cast<const f4*>(p)); }
__device__ __forceinline__ void st4_nt(float* p, f4 v) {
  __builtin_nontemporal_store(v, (P2P_GLOBAL f4*)(p));
}

template <bool NT>
__device__ __forceinline__ void st4(float* p, f4 v) {
  if (NT) st4_nt(p, v); else *reinterpret_cast<f4*>(p) = v;
}

// The whole-tile stores' cache policy (P2P_DELTA_STORE_AUX): -1 nontemporal
// global stores; else buffer stores with those cache-policy bits (bit 0
// sc0, bit 1 nt, bit 4 sc1) through a descriptor at the tile's base -- the
// A/B builds' knob (tools/variants/delta_*.py; the split kernel's w stores
// won by device-scope sc1, fedavg.hip st_w).
#ifndef P2P_DELTA_STORE_AUX
#define P2P_DELTA_STORE_AUX 16
#endif
typedef uint32_t du4 __attribute__((ext_vector_type(4)));
// v to base[off .. off + 3]: base wave-uniform, off < 2^20 floats past it.
__device__ __forceinline__ void st4_tile(float* base, uint32_t off, f4 v) {
#if P2P_DELTA_STORE_AUX < 0
  st4_nt(base + off, v);
#else
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 1u << 22, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(du4, v), rs, off * 4u, 0, P2P_DELTA_STORE_AUX);
#endif
}

// One tile of kBlock*4*NV floats (the segments kernel and the ABI's
// P2P_DELTA_TILE use NV = kDNV).
template <int NV = kDNV, bool NT = true>
__device__ __forceinline__ void delta_tile(const float* cur, float* prev, float* delta, int64_t n,
                                           int64_t tile0, bool first) {
  constexpr int kT = kBlock * 4 * NV;
  const int64_t base = tile0 + 4 * static_cast<int64_t>(threadIdx.x);
  const bool aligned =
      ((reinterpret_cast<uintptr_t>(cur) | reinterpret_cast<uintptr_t>(prev) | reinterpret_cast<uintptr_t>(delta)) &
       15) == 0;
  if (aligned && tile0 + kT <= n) {
    f4 c[NV], p[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) c[v] = ld4_nt(cur + base + kBlock * 4 * v);
    if (!first) {
#pragma unroll
      for (int v = 0; v < NV; ++v) p[v] = ld4_nt(prev + base + kBlock * 4 * v);
    }
    if (NT) {  // descriptors at the tile's base (wave-uniform): the store policy above
      float* db = reinterpret_cast<float*>(uniform_u64(reinterpret_cast<uint64_t>(delta + tile0)));
      float* pb = reinterpret_cast<float*>(uniform_u64(reinterpret_cast<uint64_t>(prev + tile0)));
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const uint32_t o = static_cast<uint32_t>(4 * threadIdx.x + kBlock * 4 * v);
        st4_tile(db, o, first ? c[v] : c[v] - p[v]);  // (:279) or the first-round copy (:275)
        st4_tile(pb, o, c[v]);                          // clone (:282)
      }
      return;
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int64_t o = base + kBlock * 4 * v;
      st4<NT>(delta + o, first ? c[v] : c[v] - p[v]);  // (:279) or the first-round copy (:275)
      st4<NT>(prev + o, c[v]);                          // clone (:282)
    }
    return;
  }
#pragma unroll 1
  for (int v = 0; v < NV; ++v)
#pragma unroll 1
    for (int e = 0; e < 4; ++e) {
      const int64_t i = base + kBlock * 4 * v + e;
      if (i >= n) continue;
      const float x = ldg(cur + i);
      stg(delta + i, first ? x : x - ldg(prev + i));
      stg(prev + i, x);
    }
}

template <int NV, bool NT>
__global__ __launch_bounds__(kBlock) void delta_flat_kernel(const float* cur, float* prev, float* delta,
                                                            int64_t n, int first) {
  delta_tile<NV, NT>(cur, prev, delta, n, static_cast<int64_t>(blockIdx.x) * (kBlock * 4 * NV), first != 0);
}

// Whole state_dict: one tile per block, segment by binary search on tile_begin.
__global__ __launch_bounds__(kBlock) void delta_segments_kernel(const p2p_delta_segment_t* __restrict__ segs,
                                                                int nseg, int first) {
  const int64_t t = blockIdx.x;
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    const int64_t tb = ldc(&segs[mid].tile_begin);
    if (tb <= t) lo = mid; else hi = mid - 1;
    lo = __builtin_amdgcn_readfirstlane(lo);
    hi = __builtin_amdgcn_readfirstlane(hi);
  }
  const p2p_delta_segment_t* sp = segs + lo;
  const float* cur = ldc(&sp->cur);
  float* prev = ldc(&sp->prev);
  float* delta = ldc(&sp->delta);
  const int64_t n = ldc(&sp->n);
  const int64_t tb = ldc(&sp->tile_begin);
  delta_tile<kDNV, true>(cur, prev, delta, n, (t - tb) * kDTile, first != 0);
}

}  // namespace p2p

using namespace p2p;

static int32_t delta_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? P2P_OK : static_cast<int32_t>(e);
}

extern "C" int32_t p2p_delta_snapshot_f32(const float* cur, float* prev, float* delta, int64_t n, int32_t first,
                                          p2p_stream_t stream) {
  if (!cur || !prev || !delta || n < 0) return P2P_ERR_INVALID;
  if ((reinterpret_cast<uintptr_t>(cur) | reinterpret_cast<uintptr_t>(prev) | reinterpret_cast<uintptr_t>(delta)) &
      3)
    return P2P_ERR_ALIGN;
  if (n == 0) return P2P_OK;
  // one float4 per lane, nontemporal loads and stores: the fastest of the
  // NV in {1, 2, 4, 8} x {plain, nontemporal} grid measured.
  const int64_t tiles = ceil_div(n, kDTile);
  if (tiles > 0x7FFFFFFFll) return P2P_ERR_UNSUPPORTED;
  hipLaunchKernelGGL((delta_flat_kernel<kDNV, true>), dim3(static_cast<unsigned>(tiles)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), cur, prev, delta, n, first);
  return delta_status();
}

extern "C" int32_t p2p_delta_snapshot_segments_f32(const p2p_delta_segment_t* segs, int32_t nseg,
                                                   int64_t total_tiles, int32_t first, p2p_stream_t stream) {
  if (!segs || nseg < 1 || total_tiles < 0) return P2P_ERR_INVALID;
  if (total_tiles > 0x7FFFFFFFll) return P2P_ERR_UNSUPPORTED;
  if (total_tiles == 0) return P2P_OK;
  hipLaunchKernelGGL(delta_segments_kernel, dim3(static_cast<unsigned>(total_tiles)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), segs, nseg, first);
  return delta_status();
}
