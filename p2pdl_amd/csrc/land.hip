// K5 device half -- landing a received update in its slab row (SURVEY.md
// §8(f) row 1; reference node/node.py:135-141 unpickles every update into
// fresh tensors, one allocation + copy per tensor).
//
// The message (the pickled state_dict, node/node.py:285) arrives in a pinned
// host buffer and crosses PCIe in ONE DMA, as bytes, into a device byte
// buffer.  This kernel then places every fp32 payload at its 256-B aligned
// offset in the slab row -- one launch per update over a segment table (one
// entry per tensor), so the host never touches the payload bytes: no staging
// memcpy, no per-tensor copy call.
//
// Payloads sit at arbitrary byte offsets inside the pickle, the row offsets
// are 4-B aligned: lane i of a tile writes float i (coalesced, 256 B per wave
// instruction) from two aligned source dwords funnel-shifted by the payload's
// byte misalignment (v_alignbyte).  Reads never pass msg_bytes: the last
// dword of a misaligned payload is assembled from bytes when its aligned
// successor would.  HBM-bound byte movement (8 B per float: 4 read, 4
// written), ~40 us for a 47 MB ResNet-18 update.
#include "p2p_common.h"

namespace p2p {

constexpr int kLandNV = P2P_LAND_TILE / kBlock;  // floats per lane per tile (16)

__device__ __forceinline__ p2p_land_segment_t load_land_segment(const p2p_land_segment_t* segs, int nseg,
                                                                int64_t t) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    const int64_t tb = ldc(&segs[mid].tile_begin);
    if (tb <= t) lo = mid; else hi = mid - 1;
    lo = __builtin_amdgcn_readfirstlane(lo);
    hi = __builtin_amdgcn_readfirstlane(hi);
  }
  const p2p_land_segment_t* sp = segs + lo;
  p2p_land_segment_t s;
  s.src_off = ldc(&sp->src_off);
  s.dst = ldc(&sp->dst);
  s.n = ldc(&sp->n);
  s.tile_begin = ldc(&sp->tile_begin);
  return s;
}

// The 4 bytes at msg + a (any alignment), reading nothing at or past msg_bytes.
__device__ __forceinline__ uint32_t load_u32_any(const uint8_t* msg, uint64_t a, uint64_t msg_bytes) {
  const uint64_t q = a & ~uint64_t(3);
  const uint32_t sh = static_cast<uint32_t>(a & 3);
  const uint32_t lo = ldg(reinterpret_cast<const uint32_t*>(msg + q));
  if (sh == 0) return lo;
  if (q + 8 <= msg_bytes) {
    const uint32_t hi = ldg(reinterpret_cast<const uint32_t*>(msg + q + 4));
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
  }
  uint32_t v = 0;  // the message's last bytes: assemble without the aligned successor
  for (uint32_t b = 0; b < 4; ++b) v |= static_cast<uint32_t>(ldg(msg + a + b)) << (8 * b);
  return v;
}

__global__ __launch_bounds__(kBlock) void land_segments_kernel(const uint8_t* __restrict__ msg, uint64_t msg_bytes,
                                                                const p2p_land_segment_t* __restrict__ segs,
                                                                int nseg, int64_t ntiles, unsigned gx) {
  const int64_t t = tile_id(gx);
  if (t >= ntiles) return;  // block-uniform
  const p2p_land_segment_t s = load_land_segment(segs, nseg, t);
  const int64_t i0 = (t - s.tile_begin) * P2P_LAND_TILE + static_cast<int64_t>(threadIdx.x);
  uint32_t v[kLandNV];
#pragma unroll
  for (int j = 0; j < kLandNV; ++j) {  // all loads first, then the stores
    const int64_t i = i0 + static_cast<int64_t>(j) * kBlock;
    const uint64_t a = s.src_off + 4 * static_cast<uint64_t>(i);
    v[j] = (i < s.n && a + 4 <= msg_bytes) ? load_u32_any(msg, a, msg_bytes) : 0u;
  }
#pragma unroll
  for (int j = 0; j < kLandNV; ++j) {
    const int64_t i = i0 + static_cast<int64_t>(j) * kBlock;
    if (i < s.n) stg(reinterpret_cast<uint32_t*>(s.dst) + i, v[j]);
  }
}

}  // namespace p2p

using namespace p2p;

extern "C" int32_t p2p_land_segments_f32(const uint8_t* msg, uint64_t msg_bytes, const p2p_land_segment_t* segs,
                                         int32_t nseg, int64_t total_tiles, p2p_stream_t stream) {
  if (!msg || !segs || nseg < 1 || total_tiles < 0) return P2P_ERR_INVALID;
  if (total_tiles == 0) return P2P_OK;
  const TileGrid tg = tile_grid(total_tiles, kBlock);
  hipLaunchKernelGGL(land_segments_kernel, dim3(tg.gx, tg.gy), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                     msg, msg_bytes, segs, nseg, total_tiles, tg.gx);
  return static_cast<int32_t>(hipGetLastError());
}
