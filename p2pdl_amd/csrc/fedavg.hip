// K1 -- streaming K-peer FedAvg reduction + apply for gfx950.
//
// Replaces reference aggregator/aggregation.py:15-38:
//   acc = zeros_like(p)                         (:15)  -> acc = +0 in registers
//   for upd in received_models: acc += upd[key]  (:25-28) -> fixed peer order
//   acc /= num_updates                           (:31-32) -> IEEE true division
//   state_dict()[key] += 0.1 * acc               (:36-38) -> mul rounded, add rounded
// P2P_RULE_FEDAVG_TORCH_GPU (RECIP below) reproduces the same ops as torch
// runs them on a GPU tensor -- the reference's own deployment, the model on
// cuda (node/node.py:28-29): ATen divides by a CPU scalar as a multiply by
// fl(1/K) (measured on MI355X, tools/torch_div_probe.py: 20-54% of elements
// differ from the true quotient at K = 3, 7, 10, 100).
//
// The reference issues K*L separate add_ kernels, each reading acc + update and
// writing acc (3x the algorithmic traffic).  Here one pass reads every peer
// element once, keeps the running sum in VGPRs and touches w once:
// algorithmic bytes = 4*n*(K+2) per launch (K peer reads + w read + w write).
//
// Layout (measured, tools/fedavg_sweep.hip): a 256-lane block owns a tile
// of NV x 1024 floats; lane l owns the float4s at l, l+256, ... of it, so
// EVERY load instruction reads one contiguous 1 KB per wave (a lane-
// contiguous 32-B layout halves the useful bytes per instruction and ran at
// 61-73% of peak).  The peer loop is unrolled 8 deep, peer streams use
// nontemporal loads (read once), one tile per block.  128 GB cfg3 tile:
// 6.2-6.4 TB/s = 78-80% of 8 TB/s.  No inter-block reuse exists, so no XCD
// remap is needed (guide T1: 0% on elementwise).
#include <atomic>

#include "p2p_common.h"

namespace p2p {

typedef float f4 __attribute__((ext_vector_type(4)));

// Four float4 per lane per peer per tile (4096 floats) for flat buffers AND
// state_dict segments: 4 x 8 independent 1-KiB wave loads in flight per lane.
// Only the full-tile path is 4-wide; the ragged last tile of a buffer runs as
// four 1024-float sub-tiles, so the kernels stay at 64 / 74 VGPRs (round 1's
// 4-wide ragged path took the segment kernel to 150 VGPRs and lost to one
// float4 per lane).  Round 2 A/B against one float4 per lane, same box
// (profiles/r02/ab/abfa4): cfg3 21.02 vs 21.25 ms, cfg2 0.518 vs 0.522 ms;
// the standalone sweep (tools/fedavg_sweep.hip) shows the same order.
constexpr int kNV = 4;
constexpr int kTile = kBlock * 4 * kNV;   // 4096 floats per tile
template <int NV> constexpr int tile_of() { return kBlock * 4 * NV; }
constexpr int kUnroll = 8;

__device__ __forceinline__ f4 ld_nt(const float* p) { return ldg_nt(reinterpret_cast<const f4*>(p)); }
__device__ __forceinline__ f4 ld(const float* p) { return ldg(reinterpret_cast<const f4*>(p)); }
__device__ __forceinline__ void st(float* p, f4 v) { stg(reinterpret_cast<f4*>(p), v); }

// acc / K (:31-32): IEEE division, or (RECIP) torch's GPU form acc * fl(1/K)
// with inv = 1.0f / K correctly rounded (-fhip-fp32-correctly-rounded-divide-sqrt).
template <bool RECIP>
__device__ __forceinline__ float div1(float a, float k, float inv) {
  return RECIP ? __fmul_rn(a, inv) : a / k;
}
template <bool RECIP>
__device__ __forceinline__ f4 div4(f4 a, float k, float inv) {
  f4 r;
  r.x = div1<RECIP>(a.x, k, inv); r.y = div1<RECIP>(a.y, k, inv);
  r.z = div1<RECIP>(a.z, k, inv); r.w = div1<RECIP>(a.w, k, inv);
  return r;
}
__device__ __forceinline__ f4 apply4(f4 w, float lr, f4 m) {
  f4 r;
  r.x = apply_lr(w.x, lr, m.x); r.y = apply_lr(w.y, lr, m.y);
  r.z = apply_lr(w.z, lr, m.z); r.w = apply_lr(w.w, lr, m.w);
  return r;
}

// One tile starting at `tile0`; this lane's part.  FULL: every float4 group
// of the tile is in range (no predicates).  !FULL (the last, ragged tile):
// complete float4 groups still use vector loads under a per-lane predicate;
// the <= 3 trailing elements of the array go element by element.  Same op
// order on every path.
template <int NV, bool FULL, bool RECIP>
__device__ __forceinline__ void fedavg_tile_vec(const float* const* __restrict__ peers, int K,
                                                int64_t n, int64_t base, float* w, float* out,
                                                float lr) {
  const float fk = static_cast<float>(K);
  const float inv = RECIP ? 1.0f / fk : 0.f;
  bool ok[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) ok[v] = FULL || (base + kBlock * 4 * v + 4 <= n);
  f4 acc[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) acc[v] = f4{0.f, 0.f, 0.f, 0.f};  // +0 init (:15)
  int k = 0;
  for (; k + kUnroll <= K; k += kUnroll) {
    f4 x[kUnroll][NV];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const float* p = table_at(peers, k + u) + base;
#pragma unroll
      for (int v = 0; v < NV; ++v)
        x[u][v] = ok[v] ? ld_nt(p + kBlock * 4 * v) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u)  // strictly in list order (:25-28)
#pragma unroll
      for (int v = 0; v < NV; ++v) acc[v] += x[u][v];
  }
  for (; k < K; ++k) {
    const float* p = table_at(peers, k) + base;
#pragma unroll
    for (int v = 0; v < NV; ++v)
      acc[v] += ok[v] ? ld_nt(p + kBlock * 4 * v) : f4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    if (!ok[v]) continue;
    const int64_t o = base + kBlock * 4 * v;
    const f4 m = div4<RECIP>(acc[v], fk, inv);  // (:31-32)
    if (out) st(out + o, m);
    if (w) st(w + o, apply4(ld(w + o), lr, m));  // (:36-38)
  }
}

// Element-wise path (misaligned views, and the < 4 trailing elements).
template <bool RECIP>
__device__ __forceinline__ void fedavg_elem(const float* const* __restrict__ peers, int K, int64_t i,
                                            float* w, float* out, float lr) {
  float acc = 0.f;
#pragma unroll 8
  for (int k = 0; k < K; ++k) acc += ldg(table_at(peers, k) + i);
  const float fk = static_cast<float>(K);
  const float m = div1<RECIP>(acc, fk, RECIP ? 1.0f / fk : 0.f);
  if (out) stg(out + i, m);
  if (w) stg(w + i, apply_lr(ldg(w + i), lr, m));
}

// Element-wise over E coordinates per lane at once -- first + stride * j, j
// < E, those below n -- for views that are only 4-B aligned: every load
// instruction still reads one contiguous 256 B per wave, and the lane keeps
// E x U loads in flight where one coordinate at a time kept 8 (K = 256 over
// 1.8M coordinates of 8-B aligned rows: 0.18 of HBM peak that way,
// tools/grid_ab.py).  Each coordinate sums its peers in list order from +0.
// The VGPR kernels take 8 coordinates x 2 peers per pass: their aligned
// path's register budget (74 VGPRs) holds, where 16 x 4 took them to 134
// for the same misaligned rate (0.66 of peak at K = 8, tools/vgpr_ab.py).
template <int E, bool RECIP, int U = 4>
__device__ __forceinline__ void fedavg_scalar(const float* const* __restrict__ peers, int K, int64_t n,
                                              int64_t first, int stride, float* w, float* out, float lr) {
  bool ok[E];
#pragma unroll
  for (int j = 0; j < E; ++j) ok[j] = first + static_cast<int64_t>(stride) * j < n;
  float acc[E];
#pragma unroll
  for (int j = 0; j < E; ++j) acc[j] = 0.f;  // +0 init (:15)
  int k = 0;
  for (; k + U <= K; k += U) {
    float x[U][E];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float* p = table_at(peers, k + u) + first;
#pragma unroll
      for (int j = 0; j < E; ++j) x[u][j] = ok[j] ? ldg_nt(p + static_cast<int64_t>(stride) * j) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)  // strictly in list order (:25-28)
#pragma unroll
      for (int j = 0; j < E; ++j) acc[j] += x[u][j];
  }
  for (; k < K; ++k) {
    const float* p = table_at(peers, k) + first;
#pragma unroll
    for (int j = 0; j < E; ++j) acc[j] += ok[j] ? ldg_nt(p + static_cast<int64_t>(stride) * j) : 0.f;
  }
  const float fk = static_cast<float>(K);
  const float inv = RECIP ? 1.0f / fk : 0.f;
#pragma unroll
  for (int j = 0; j < E; ++j) {
    if (!ok[j]) continue;
    const int64_t i = first + static_cast<int64_t>(stride) * j;
    const float m = div1<RECIP>(acc[j], fk, inv);  // (:31-32)
    if (out) stg(out + i, m);
    if (w) stg(w + i, apply_lr(ldg(w + i), lr, m));  // (:36-38)
  }
}

template <int NV, bool RECIP>
__device__ __forceinline__ void fedavg_tile(const float* const* __restrict__ peers, int K,
                                            int64_t n, int64_t tile0, float* w, float* out,
                                            float lr, bool aligned) {
  const int64_t base = tile0 + 4 * static_cast<int64_t>(threadIdx.x);
  if (aligned) {
    if (tile0 + tile_of<NV>() <= n) {
      fedavg_tile_vec<NV, true, RECIP>(peers, K, n, base, w, out, lr);
      return;
    }
    // ragged last tile: 1024-float sub-tiles (same per-element op order)
#pragma unroll 1
    for (int v = 0; v < NV; ++v) {
      const int64_t g = base + kBlock * 4 * v;
      if (tile0 + kBlock * 4 * v >= n) break;
      fedavg_tile_vec<1, false, RECIP>(peers, K, n, g, w, out, lr);
      if (g < n && g + 4 > n)  // trailing elements of a float4 group that straddles n
        for (int64_t i = g; i < n; ++i) fedavg_elem<RECIP>(peers, K, i, w, out, lr);
    }
    return;
  }
  // 8 coordinates per lane per pass (the tile's 4 * NV in passes): the
  // vector path's register budget holds (64 / 74 VGPRs, occupancy 8 / 6)
  if constexpr (NV == 1) {
    fedavg_scalar<4, RECIP, 2>(peers, K, n, tile0 + threadIdx.x, kBlock, w, out, lr);
  } else {
#pragma unroll 1
    for (int h = 0; h < NV / 2; ++h)
      fedavg_scalar<8, RECIP, 2>(peers, K, n, tile0 + threadIdx.x + h * 8 * kBlock, kBlock, w, out, lr);
  }
}

// Flat buffer, one tile per block, tiles tile_base, tile_base + 1, ...  K
// either from the kernarg or, when k_dev != nullptr, from device memory
// (fused accept -> FedAvg path).
template <int NV, bool RECIP>
__global__ __launch_bounds__(kBlock) void fedavg_flat_kernel(const float* const* __restrict__ peers,
                                                             int K, const int32_t* k_dev,
                                                             int64_t n, float* w, float* out,
                                                             float lr, int64_t tile_base) {
  if (k_dev) K = *k_dev;
  if (K <= 0) return;
  const bool aligned = all_aligned16(peers, K, w, out);
  fedavg_tile<NV, RECIP>(peers, K, n, (tile_base + static_cast<int64_t>(blockIdx.x)) * tile_of<NV>(), w, out, lr,
                         aligned);
}

// ---------------------------------------------------------------------------
// K1s (round 5): the same reduction with the peer streams staged by LDS-DMA
// through DEDICATED loader waves (tools/fedavg_split.hip, profiles/r05/split*).
//
// A block = kSL loader waves + kSC consumer waves and owns tiles b, b + G, ...
// of kSTile floats.  A stage is one peer's 32-KiB slice of one tile; the
// block's stages run (tile, peer) in list order through a ring of kSS
// stages in LDS (+ one slot for the tile's w).  Loaders issue
// global_load_lds_dwordx4 nt (1 KiB per wave instruction, no VGPR
// destination); one barrier per stage: before barrier i each loader waits
// (vmcnt) for its part of stage i, after it refills the slot stage i-1 used
// with stage i + kSS - 1, so 1-2 stages (32-64 KiB) are in flight per CU at
// every moment beside the one the consumers read.
// Consumer wave c owns floats [c * kSTile / kSC, (c + 1) * kSTile / kSC) of
// the tile: ds_read_b128 of its part of stage i and the add, in peer order
// from +0 (:15, :25-28); after the tile's last peer / K and the apply
// (:31-38) exactly as fedavg_tile_vec -- the same per-coordinate op order,
// so the bits are those of the VGPR kernel.  128 KiB of LDS per block (3
// stages + w) leaves a third of the CU's LDS to a kernel running beside it
// (RCCL's all-gather at N > 1).  Measured against the VGPR
// kernel, interleaved on one box: cfg3 tile (256 x 125M) +2-3%, 256 x 16M
// +2-7% across three boxes; the loaders alone (no consumers) reach 6.4-7.0
// TB/s with this access pattern.
constexpr int kSL = 4;                       // loader waves
constexpr int kSC = 8;                       // consumer waves
#ifndef P2P_SPLIT_STAGES
#define P2P_SPLIT_STAGES 3  // (an A/B build may set 4: 160 KiB of LDS)
#endif
constexpr int kSS = P2P_SPLIT_STAGES;        // ring stages (+ w: 128 KiB of LDS)
constexpr int kSTile = 8192;                 // floats per tile (32 KiB per peer)
constexpr int kSPer = kSTile / 256 / kSL;    // DMA instructions per loader per stage
constexpr int kSRpw = kSTile / 256 / kSC;    // ds_read_b128 per consumer lane per stage
static_assert((kSS - 2) * kSPer <= 63, "vmcnt is 6 bits");
static_assert(kSRpw == 4, "lds_read4");
constexpr int kSplitMinK = 16;

#define P2P_LDS __attribute__((address_space(3)))
template <int AUX>
__device__ __forceinline__ void dma16(const float* src, float* lds_dst) {
  __builtin_amdgcn_global_load_lds((P2P_GLOBAL void*)(const_cast<float*>(src)), (P2P_LDS void*)lds_dst, 16, 0, AUX);
}
// The split kernel's w path: the w slice DMA'd into LDS beside the stages
// (cache policy P2P_W_DMA_AUX: 0 plain, 2 nontemporal) and the epilogue's w /
// out stores (P2P_W_STORE_AUX: -1 plain global stores; else buffer stores
// with those cache-policy bits -- bit 0 sc0, bit 1 nt, bit 4 sc1).  Same
// bits either way.  The stores were the split kernel's per-tile cost: the
// lab's queue kernel with its w stores dropped runs 4-14% faster at K = 64 /
// 16 while dropping the w DMA alone changes ~1% (tools/split_fixed_lab.hip
// probes, profiles/r06/wpath).  Device-scope (sc1) stores, written through
// the XCD's L2 instead of lingering there dirty among the peer stream, with
// the w DMA nontemporal: same process, launch by launch against plain
// stores (tools/lib_pair_ab.py, tools/variants/wpath_*.py): K = 256 x 16.8M
// +1.1%, 64 x 100M +2.1%, 16 x 11.7M +2.1%, 16 x 100M +3.6%, the cfg2 rows
// kernel +1.0%, the chunk list +1.3% -- the best of nt / sc0 sc1 / sc1 nt /
// sc0 sc1 nt.
#ifndef P2P_W_DMA_AUX
#define P2P_W_DMA_AUX 2
#endif
#ifndef P2P_W_STORE_AUX
#define P2P_W_STORE_AUX 16
#endif
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
// v to base[off .. off + 3]: base wave-uniform, off < kSTile (a tile's or a
// chunk's floats past base).
__device__ __forceinline__ void st_w(float* base, uint32_t off, f4 v) {
#if P2P_W_STORE_AUX < 0
  st(base + off, v);
#else
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, kSTile * 4, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), rs, off * 4u, 0, P2P_W_STORE_AUX);
#endif
}

// Four ds_read_b128 of this lane's part at LDS byte address a, waited in the
// same statement (hipcc neither counts nor reorders around it).
__device__ __forceinline__ void lds_read4(f4 (&x)[4], uint32_t a) {
  asm volatile(
      "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:1024\n\t"
      "ds_read_b128 %2, %4 offset:2048\n\tds_read_b128 %3, %4 offset:3072\n\ts_waitcnt lgkmcnt(0)"
      : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3])
      : "v"(a));
}

// Where split tile t lives: a flat buffer (tile t at t * kSTile), or (SEGS)
// entry t of a host-built tile list naming a segment of a state_dict table
// and the tile's first element in it.  Wave-uniform (scalar loads).
struct SplitTile {
  const float* const* peers;
  float* w;
  float* out;
  int64_t c0;
};
template <bool SEGS>
__device__ __forceinline__ SplitTile split_tile(const float* const* peers, float* w, float* out,
                                                const p2p_split_tile_t* tiles, const Seg* segs, int64_t t) {
  if constexpr (SEGS) {
    const int64_t seg = ldc(&tiles[t].seg);
    const int64_t c0 = ldc(&tiles[t].c0);
    const Seg* sp = segs + seg;
    return SplitTile{ldc(&sp->peers), ldc(&sp->w), ldc(&sp->out), c0};
  } else {
    return SplitTile{peers, w, out, t * kSTile};
  }
}

// The consumer side of one tile: K stages added in peer order from +0 (:15,
// :25-28), one barrier per stage; `hook(k)` runs right after barrier k (the
// tile queue's publication, QUEUE below; a no-op otherwise).
template <typename Hook>
__device__ __forceinline__ void sum_stages(f4 (&acc)[kSRpw], int K, uint32_t lds0, uint32_t mine, int& slot,
                                           Hook&& hook) {
#pragma unroll
  for (int r = 0; r < kSRpw; ++r) acc[r] = f4{0.f, 0.f, 0.f, 0.f};  // +0 init (:15)
  for (int k = 0; k < K; ++k) {
    __builtin_amdgcn_s_barrier();
    hook(k);
    f4 x[kSRpw];
    lds_read4(x, lds0 + static_cast<uint32_t>(slot) * (kSTile * 4) + mine);
#pragma unroll
    for (int r = 0; r < kSRpw; ++r) acc[r] += x[r];  // strictly in list order (:25-28)
    slot = slot + 1 == kSS ? 0 : slot + 1;
  }
}

// One ROWS tile of consumer wave cw: its chunk's w slice DMA'd beside the
// stages (lanes inside the chunk's valid floats only), the K stages added in
// peer order, then / K and the apply where the chunk holds model floats --
// element-wise for the float4 that straddles the key's end.
template <bool RECIP, typename Hook>
__device__ __forceinline__ void rows_tile(const p2p_row_chunk_t* ch, int K, int lane, float lr, float fk, float inv,
                                          float* lds, uint32_t lds0, uint32_t mine, int& slot, int cw, Hook&& hook) {
  float* cwp = ldc(&ch->w);
  const int64_t valid = ldc(&ch->valid);
  if (cwp) {
#pragma unroll
    for (int r = 0; r < kSRpw; ++r) {
      const int idx = lane * 4 + r * 256;
      if (idx + 4 <= valid) dma16<P2P_W_DMA_AUX>(cwp + idx, &lds[kSS * kSTile + (cw * kSRpw + r) * 256]);
    }
  }
  f4 acc[kSRpw];
  sum_stages(acc, K, lds0, mine, slot, hook);
  if (!cwp) return;  // padding between keys: averaged, dropped
  f4 m[kSRpw];
#pragma unroll
  for (int r = 0; r < kSRpw; ++r) m[r] = div4<RECIP>(acc[r], fk, inv);  // (:31-32)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's w DMA (and its older stores)
  f4 wq[kSRpw];
  lds_read4(wq, lds0 + static_cast<uint32_t>(kSS * kSTile * 4) + mine);
#pragma unroll
  for (int r = 0; r < kSRpw; ++r) {
    const int idx = lane * 4 + r * 256;
    if (idx + 4 <= valid) {
      st_w(cwp, idx, apply4(wq[r], lr, m[r]));  // (:36-38)
    } else if (idx < valid) {  // the key's last, partial float4
      const float mv[4] = {m[r].x, m[r].y, m[r].z, m[r].w};
      for (int e = 0; idx + e < valid; ++e) stg(cwp + idx + e, apply_lr(ldg(cwp + idx + e), lr, mv[e]));
    }
  }
}

// CHUNKS (round 6): a state_dict of separately allocated tensors -- the
// reference caller's pickle.loads dicts (node/node.py:138-141) -- in ONE
// launch.  Split tile t is the 8 chunks list[8t .. 8t + 7]; chunk c names
// segment seg (-1: padding) and its first element c0, and holds the
// segment's floats [c0, c0 + valid), valid = min(1024, n - c0).  Loader wave
// wv streams chunks 2wv and 2wv + 1 of each stage, each from its own key's
// peer pointer, through a buffer descriptor whose range ends at the chunk's
// last whole float4: the lanes past it issue no memory request (an
// out-of-range buffer access), every wave still issues exactly kSPer DMAs
// per stage (the vmcnt arithmetic holds), and no read leaves a tensor.
// Consumer wave c owns chunk c of the tile, as in ROWS; the one float4 that
// straddles a key's end (n % 4 != 0) is summed element by element from the
// peers in list order (the same op order as fedavg_elem).
struct ChunkSrc {
  const float* const* peers;  // the key's K peer pointers (nullptr: padding)
  int64_t c0;                 // the chunk's first element in the key
  uint32_t bytes;             // the DMA range: the chunk's whole float4s, in bytes
};
__device__ __forceinline__ ChunkSrc chunk_src(const p2p_split_tile_t* list, const Seg* segs, int64_t c) {
  const int64_t seg = ldc(&list[c].seg);
  if (seg < 0) return ChunkSrc{nullptr, 0, 0u};
  const int64_t c0 = ldc(&list[c].c0);
  const Seg* sp = segs + seg;
  const int64_t n = ldc(&sp->n);
  const int64_t valid = n - c0 < P2P_ROW_CHUNK ? n - c0 : P2P_ROW_CHUNK;
  return ChunkSrc{ldc(&sp->peers), c0, static_cast<uint32_t>((valid & ~int64_t(3)) * 4)};
}
constexpr int kChunkDma = P2P_ROW_CHUNK / 256;  // 1-KiB DMAs per chunk per stage
static_assert(kSPer == 2 * kChunkDma, "a loader wave streams two chunks per stage");
// Peer ki's part of chunk cs into LDS float offset `dst`: kChunkDma buffer
// DMAs (nt), lanes past the range masked by the descriptor.  A padding chunk
// gets an empty range over a valid base (the list itself): no request at all.
__device__ __forceinline__ void chunk_dma(const ChunkSrc& cs, int ki, const void* any, float* dst, int lane) {
  const float* src = cs.bytes ? table_at(cs.peers, ki) + cs.c0 : static_cast<const float*>(any);
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), 0, cs.bytes, 0x00020000);
#pragma unroll
  for (int q = 0; q < kChunkDma; ++q)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (P2P_LDS void*)(dst + q * 256), 16, (q * 256 + lane * 4) * 4, 0, 0,
                                             2 /* nt */);
}

// One CHUNKS tile of consumer wave cw (see above).
template <bool RECIP, typename Hook>
__device__ __forceinline__ void chunks_tile(const p2p_split_tile_t* list, const Seg* segs, int64_t c, int K, int lane,
                                            float lr, float fk, float inv, float* lds, uint32_t lds0, uint32_t mine,
                                            int& slot, int cw, Hook&& hook) {
  const int64_t seg = ldc(&list[c].seg);
  const float* const* cp = nullptr;
  float *cwp = nullptr, *cop = nullptr;
  int64_t c0 = 0, valid = 0;
  if (seg >= 0) {
    const Seg* sp = segs + seg;
    c0 = ldc(&list[c].c0);
    const int64_t n = ldc(&sp->n);
    valid = n - c0 < P2P_ROW_CHUNK ? n - c0 : P2P_ROW_CHUNK;
    cp = ldc(&sp->peers);
    float* wb = ldc(&sp->w);
    float* ob = ldc(&sp->out);
    cwp = wb ? wb + c0 : nullptr;
    cop = ob ? ob + c0 : nullptr;
  }
  if (cwp) {
#pragma unroll
    for (int r = 0; r < kSRpw; ++r) {
      const int idx = lane * 4 + r * 256;
      if (idx + 4 <= valid) dma16<P2P_W_DMA_AUX>(cwp + idx, &lds[kSS * kSTile + (cw * kSRpw + r) * 256]);
    }
  }
  f4 acc[kSRpw];
  sum_stages(acc, K, lds0, mine, slot, hook);
  if (valid <= 0) return;  // padding
  f4 m[kSRpw];
#pragma unroll
  for (int r = 0; r < kSRpw; ++r) m[r] = div4<RECIP>(acc[r], fk, inv);  // (:31-32)
  if (cop) {
#pragma unroll
    for (int r = 0; r < kSRpw; ++r)
      if (lane * 4 + r * 256 + 4 <= valid) st_w(cop, lane * 4 + r * 256, m[r]);
  }
  if (cwp) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's w DMA (and its older stores)
    f4 wq[kSRpw];
    lds_read4(wq, lds0 + static_cast<uint32_t>(kSS * kSTile * 4) + mine);
#pragma unroll
    for (int r = 0; r < kSRpw; ++r)
      if (lane * 4 + r * 256 + 4 <= valid) st_w(cwp, lane * 4 + r * 256, apply4(wq[r], lr, m[r]));  // (:36-38)
  }
  if (valid & 3) {  // the key's last, partial float4: its lane sums it from the peers themselves
    const int idx = static_cast<int>(valid & ~int64_t(3));
    if (lane == (idx & 255) >> 2) {
      float* wq = cwp ? cwp - c0 : nullptr;
      float* oq = cop ? cop - c0 : nullptr;
      for (int64_t i = c0 + idx; i < c0 + valid; ++i) fedavg_elem<RECIP>(cp, K, i, wq, oq, lr);
    }
  }
}

// One FLAT / SEGS tile of consumer wave cw: the w slice DMA'd beside the
// stages, the K stages, / K, the mean stored (out) and the apply (w).
template <bool RECIP, typename Hook>
__device__ __forceinline__ void flat_tile(const SplitTile& tl, int K, int lane, float lr, float fk, float inv,
                                          float* lds, uint32_t lds0, uint32_t mine, int& slot, int cw, Hook&& hook) {
  const int64_t o = tl.c0 + cw * kSRpw * 256 + lane * 4;
  const uint32_t oi = static_cast<uint32_t>(cw * kSRpw * 256 + lane * 4);  // o - tl.c0
  if (tl.w) {
#pragma unroll
    for (int r = 0; r < kSRpw; ++r)
      dma16<P2P_W_DMA_AUX>(tl.w + o + r * 256, &lds[kSS * kSTile + (cw * kSRpw + r) * 256]);
  }
  f4 acc[kSRpw];
  sum_stages(acc, K, lds0, mine, slot, hook);
  f4 m[kSRpw];
#pragma unroll
  for (int r = 0; r < kSRpw; ++r) m[r] = div4<RECIP>(acc[r], fk, inv);  // (:31-32)
  if (tl.out) {
    float* ob = reinterpret_cast<float*>(uniform_u64(reinterpret_cast<uint64_t>(tl.out + tl.c0)));
#pragma unroll
    for (int r = 0; r < kSRpw; ++r) st_w(ob, oi + r * 256, m[r]);
  }
  if (tl.w) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's w DMA (and its older stores)
    f4 wq[kSRpw];
    lds_read4(wq, lds0 + static_cast<uint32_t>(kSS * kSTile * 4) + mine);
    float* wb = reinterpret_cast<float*>(uniform_u64(reinterpret_cast<uint64_t>(tl.w + tl.c0)));
#pragma unroll
    for (int r = 0; r < kSRpw; ++r) st_w(wb, oi + r * 256, apply4(wq[r], lr, m[r]));  // (:36-38)
  }
}

// The kernel's modes.  FLAT: a flat buffer, tile t at t * kSTile (the host
// takes whole tiles).  SEGS: the host lists only whole tiles of segments
// whose K peer pointers and w / out are all 16-B aligned (ops.py checks them
// when it builds the list); a flat buffer is checked here.
// ROWS (round 5): the peers are the K rows of a state_dict slab (DeviceInbox)
// read as flat buffers -- every tile a whole one -- and the model is
// scattered: consumer wave c of tile t applies to chunks[8t + c], the w
// tensor (if any) holding the row's floats [1024(8t + c), +1024) and how
// many of them it holds (keys start on 1024-float boundaries; the padding
// between them is averaged and dropped).  The host checks the alignment.
// CHUNKS: `tiles` is the chunk list (8 entries per tile), see above; the
// host checks the alignment of every listed key.
enum SplitMode { kFlat = 0, kSegs = 1, kRows = 2, kChunks = 3 };

// QUEUE (round 6, tools/split_fixed_lab.hip variant Q): a persistent grid
// of min(tiles, CUs) blocks that claim their tiles from a counter pair of
// g_tile_queue ([claims, blocks done], zero at launch start) instead of one
// block per tile.  A block's loaders then stream tile j+1's first stages
// during tile j's epilogue (w DMA wait, / K, apply, stores), which a
// one-tile block leaves the CU idle for.  Consumer wave 0 claims the next
// tile (a vector atomic) late in the current tile and publishes it in LDS
// a few barriers later; every wave reads it after a later barrier (loaders)
// or after the tile (consumers), so the loaders know the next tile -- or
// that there is none: the same barrier count on both sides -- before its
// first stage is due (the schedule below).  The last block to finish zeroes
// the counter for the stream's next launch.
constexpr int kQW = 2, kQR = 4;
// The claim schedule.  LATE (the product): claim the next tile after barrier
// K - 8 of the current one, publish it after K - 5, the loaders read it
// after K - 4 -- a tile is reserved for ~8 stages (~10 us) before its block
// starts it (K >= 8 needed).  Early (P2P_QUEUE_LATE 0, an A/B build): claim
// at the tile's start, publish after barrier kQW, read after kQR -- a tile
// reserved for a whole tile time (~300 us at K = 256), which left the last
// tiles of a launch waiting on busy blocks while others idled.  Same
// process, alternated launch by launch (profiles/r06/pair_ab/
// pair_ab_box8_qlate.log): late against early at K = 256 x 16.8M +0.7%,
// 16 x 100M +1.3%, cfg2 rows +1.7%, chunk list +1.4%.
#ifndef P2P_QUEUE_LATE
#define P2P_QUEUE_LATE 1
#endif
constexpr int kQueueMinK = P2P_QUEUE_LATE ? 8 : kQR + kSS;  // K the queue's publication schedule needs
constexpr int kQueueMaxK = 256;        // above it one block per tile (see queue_mode)
constexpr int kAllTilesMaxK = 128;     // above it whole CU rounds even when queued (see split_tiles_for)
constexpr int kQueueSlots = 4096;      // counter pairs, one per launch in flight (see launch_split)
__device__ int32_t g_tile_queue[2 * kQueueSlots];

template <bool RECIP, int MODE, bool QUEUE = false>
__global__ __launch_bounds__(64 * (kSL + kSC)) void fedavg_split_kernel(const float* const* __restrict__ peers,
                                                                        int K, const int32_t* k_dev,
                                                                        int64_t ntiles, float* w, float* out,
                                                                        float lr, const p2p_split_tile_t* tiles,
                                                                        const Seg* segs,
                                                                        const p2p_row_chunk_t* chunks = nullptr,
                                                                        int queue_slot = -1) {
  constexpr bool SEGS = MODE == kSegs;
  __shared__ __attribute__((aligned(16))) float lds[(kSS + 1) * kSTile];
  __shared__ int64_t tq[4];
  if (k_dev) K = __builtin_amdgcn_readfirstlane(ldg(k_dev));
  if (K <= 0) return;
  const int64_t G = gridDim.x, b = bid_x();
  const int wv = __builtin_amdgcn_readfirstlane(tid_x() >> 6), lane = tid_x() & 63;
  if (MODE == kFlat && !all_aligned16(peers, K, w, out)) {
    // 4-B-aligned views: element-wise, same op order, no LDS (block-uniform)
    constexpr int kT = 64 * (kSL + kSC);
    for (int64_t t = b; t < ntiles; t += G)  // 11 x 768 >= 8192: the tile's end bounds the last
      fedavg_scalar<(kSTile + kT - 1) / kT, RECIP>(peers, K, (t + 1) * kSTile, t * kSTile + tid_x(), kT, w, out, lr);
    return;
  }
  if (wv < kSL) {
    // stages (= barriers) of this block: known up front for a static tile
    // set (b, b + G, ...); grown tile by tile from the queue otherwise
    int64_t N = QUEUE ? K : (ntiles - b + G - 1) / G * K;
    int64_t ti = b, tnext = ntiles, issued = 0;
    int ki = 0, si = 0, kb = 0, jb = 0;  // barrier k of the block's tile jb
    SplitTile tl{};
    ChunkSrc c0{}, c1{};
    auto issue = [&]() {
      if (ki == 0) {  // a new tile
        if (issued > 0) ti = QUEUE ? tnext : ti + G;
        if constexpr (MODE == kChunks) {
          c0 = chunk_src(tiles, segs, ti * kSC + 2 * wv);
          c1 = chunk_src(tiles, segs, ti * kSC + 2 * wv + 1);
        } else {
          tl = split_tile<SEGS>(peers, w, out, tiles, segs, ti);
        }
      }
      float* dst = &lds[si * kSTile + wv * kSPer * 256];
      if constexpr (MODE == kChunks) {
        chunk_dma(c0, ki, tiles, dst, lane);
        chunk_dma(c1, ki, tiles, dst + kChunkDma * 256, lane);
      } else {
        const float* src = table_at(tl.peers, ki) + tl.c0 + (wv * kSPer) * 256 + lane * 4;
#pragma unroll
        for (int q = 0; q < kSPer; ++q) dma16<2 /* nt */>(src + q * 256, dst + q * 256);
      }
      ++issued;
      si = si + 1 == kSS ? 0 : si + 1;
      if (++ki == K) ki = 0;
    };
    for (int d = 0; d < kSS - 1 && issued < N; ++d) issue();
    for (int64_t i = 0; i < N; ++i) {
      if (i + kSS - 2 < N) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((kSS - 2) * kSPer) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // stage i landed; stage i-1's slot read
      if constexpr (QUEUE) {
        if (kb == (P2P_QUEUE_LATE ? K - 4 : kQR)) {  // the block's next tile, published after barrier kQW of this one
          tnext = static_cast<int64_t>(uniform_u64(static_cast<uint64_t>(tq[(jb + 1) & 3])));
          if (tnext < ntiles) N += K;
        }
        if (++kb == K) { kb = 0; ++jb; }
      }
      if (issued < N) issue();  // into that slot
    }
    return;
  }
  const int cw = wv - kSL;
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(&lds[0]));
  const uint32_t mine = static_cast<uint32_t>(cw * kSRpw * 256 + lane * 4) * 4u;
  const float fk = static_cast<float>(K);
  const float inv = RECIP ? 1.0f / fk : 0.f;
  int slot = 0;
  auto tile = [&](int64_t t, auto&& hook) {
    if constexpr (MODE == kRows)
      rows_tile<RECIP>(chunks + t * kSC + cw, K, lane, lr, fk, inv, lds, lds0, mine, slot, cw, hook);
    else if constexpr (MODE == kChunks)
      chunks_tile<RECIP>(tiles, segs, t * kSC + cw, K, lane, lr, fk, inv, lds, lds0, mine, slot, cw, hook);
    else
      flat_tile<RECIP>(split_tile<SEGS>(peers, w, out, tiles, segs, t), K, lane, lr, fk, inv, lds, lds0, mine, slot,
                       cw, hook);
  };
  if constexpr (!QUEUE) {
    for (int64_t t = b; t < ntiles; t += G) tile(t, [](int) {});
    return;
  } else {
    int32_t* queue = g_tile_queue + 2 * queue_slot;
    int64_t t = b;
    for (int j = 0;; ++j) {
      int64_t claim = 0;
      if (!P2P_QUEUE_LATE && cw == 0 && lane == 0) claim = G + atomicAdd(&queue[0], 1);
      tile(t, [&](int k) {
        if (P2P_QUEUE_LATE && k == K - 8 && cw == 0 && lane == 0) claim = G + atomicAdd(&queue[0], 1);
        if (k == (P2P_QUEUE_LATE ? K - 5 : kQW) && cw == 0) {
          if (lane == 0) tq[(j + 1) & 3] = claim;
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
      });
      t = static_cast<int64_t>(uniform_u64(static_cast<uint64_t>(tq[(j + 1) & 3])));
      if (t >= ntiles) break;
    }
    if (cw == 0 && lane == 0 && atomicAdd(&queue[1], 1) == static_cast<int>(G) - 1) {
      atomicExch(&queue[0], 0);  // every block has made its last claim: the stream's next launch starts at 0
      atomicExch(&queue[1], 0);
    }
  }
}

// Whole state_dict: one tile per block, segment found by binary search.
// QUARTERS: a table of fewer tiles than the chip has CUs (the reference's
// MNIST MLP: 134) runs four blocks per tile, each a quarter (one float4 per
// lane per peer), so the launch covers the chip; the table is the same.
template <bool RECIP, bool QUARTERS = false>
__global__ __launch_bounds__(kBlock) void fedavg_segments_kernel(const Seg* __restrict__ segs,
                                                                 int nseg, int K, float lr) {
  const int64_t t = QUARTERS ? blockIdx.x >> 2 : blockIdx.x;
  const Seg s = load_segment(segs, nseg, t);
  const bool aligned = all_aligned16(s.peers, K, s.w, s.out);
  if constexpr (QUARTERS)
    fedavg_tile<1, RECIP>(s.peers, K, s.n, (t - s.tile_begin) * kTile + (blockIdx.x & 3) * tile_of<1>(), s.w, s.out,
                          lr, aligned);
  else
    fedavg_tile<kNV, RECIP>(s.peers, K, s.n, (t - s.tile_begin) * kTile, s.w, s.out, lr, aligned);
}

__global__ __launch_bounds__(kBlock) void apply_kernel(float* w, const float* agg, float lr,
                                                       int64_t n) {
  const bool aligned = ((reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(agg)) & 15) == 0;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock * 4;
  for (int64_t i = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) * 4; i < n; i += stride) {
    if (aligned && i + 4 <= n) {
      st(w + i, apply4(ld(w + i), lr, ld(agg + i)));
    } else {
      for (int64_t j = i; j < n && j < i + 4; ++j) stg(w + j, apply_lr(ldg(w + j), lr, ldg(agg + j)));
    }
  }
}

static int grid_for_tiles(int64_t ntiles) { return static_cast<int>(ntiles > 0 ? ntiles : 1); }

// Compute units of the current device (cached per device id; concurrent
// first calls store the same value).  Only the launch plan depends on it.
static int device_cus() {
  static std::atomic<int> cus[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  int c = cus[dev].load(std::memory_order_relaxed);
  if (c == 0) {
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
    cus[dev].store(c, std::memory_order_relaxed);
  }
  return c;
}

// Flat launches.  With K >= kSplitMinK the split kernel takes whole ROUNDS of
// kSTile tiles -- a multiple of the CU count, one block resident per CU, so
// every CU gets the same number of 32-KiB x K tiles -- and the VGPR kernel
// the rest (fewer than one tile per CU, plus the ragged tail), in 4096-float
// tiles that many blocks share per CU: 1907 tiles (a cfg3 chunk at 8 GPUs) as
// 8 split rounds would leave half the CUs idle in the last one.  K is the
// kernarg or, for the device-K path, k_max.
// Split tiles for `full` whole tiles: whole rounds of the CU count (0 below
// one round or for K < kSplitMinK) -- or, for the tile queue (`all`), every
// whole tile from one round up: its persistent blocks balance any tile count
// dynamically, and the VGPR remainder of a partial round cost more than the
// split kernel's own last claims (same process, profiles/r06/pair_ab: 64 /
// 16 x 11.7M +3.0% / +5.7%, 64 / 16 x 100M +0.2% / +0.3%).
static int64_t split_tiles_for(int K, int64_t full, bool all = false) {
  if (K < kSplitMinK || full <= 0) return 0;
  const int64_t cus = device_cus();
  if (all) return full >= cus ? full : 0;
  return full / cus * cus;
}
// One block per tile: one block is resident per CU (128 KiB of LDS), so the
// dispatcher hands each CU its next tile as it frees -- no block owns a
// fixed share of a launch, which a prime round count made one block per CU
// (59 rounds for a cfg3 tile).  Same-box A/B (tools/grid_ab.py,
// profiles/r05/grid): never slower than CUs x R blocks of equal tiles, +0.6%
// at 256 x 125M, +2.3% at 16 x 100M.
static dim3 split_grid(int64_t tiles) { return dim3(static_cast<unsigned>(tiles)); }

// QUEUE launches (see fedavg_split_kernel): launch i takes counter pair
// i mod (kQueueSlots - kQueueCaptured) of g_tile_queue (zero at module load;
// each launch leaves its pair zeroed when its last block ends).  Nothing is
// allocated and no per-stream state kept, so the call stays graph-capturable.
// A pair is reused kQueueSlots - kQueueCaptured launches later: the bound is
// that many split launches in flight at once on one device.  A launch
// captured into a graph keeps its pair for every replay, so it takes one of
// the last kQueueCaptured pairs, never handed out again (its replays run in
// order: a graph exec does not run concurrently with itself); were it to
// take a rotating pair, an ordinary launch on another stream would share it
// every 3,072 launches and, overlapping a replay, both would claim tiles from
// one counter -- each skipping the other's.  Captures past kQueueCaptured
// launch one block per tile (same results).
// Which launches take the queue: 8 <= K <= kQueueMaxK, every mode.  Same
// process, the builds alternated launch by launch on the same buffers
// (tools/lib_pair_ab.py, profiles/r06/pair_ab), against one block per tile:
// flat buffers at K = 16 / 64 +7.8% / +2.5%, chunk-list state_dicts +3.0%,
// the rows kernel (cfg2 landed) +3.5%, the K = 256 cfg3 planes +1.1% (late
// claims; with early ones the K = 256 planes lost up to 2%, and the queue
// stopped at K = 128 for a while).  (Process-level A/Bs had credited the
// queue with +3% at K = 256 and debited the rows kernel 1%: the first
// process of a pair ran faster whichever build it was,
// profiles/r06/queue_ab/README.md.)  An A/B build may set P2P_SPLIT_QUEUE 0
// (no queue at all).
#ifndef P2P_SPLIT_QUEUE
#define P2P_SPLIT_QUEUE 1
#endif
template <int MODE>
constexpr bool queue_mode() {
  return P2P_SPLIT_QUEUE && MODE >= kFlat;
}
// Does a launch take the queue: its mode, no share hint, K from the kernarg,
// long enough for the queue's publication schedule and at most kQueueMaxK.
template <int MODE>
static bool use_queue(bool share, const int32_t* k_dev, int K) {
  return queue_mode<MODE>() && !share && !k_dev && K >= kQueueMinK && K <= kQueueMaxK;
}
constexpr int kQueueCaptured = 1024;
static std::atomic<uint64_t> g_queue_next{0};  // 64-bit: i mod 3,072 never jumps at a wrap
static std::atomic<uint32_t> g_queue_captured{0};
// The counter pair of a queued launch on `st`, or -1: launch without the queue.
static int queue_slot(hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
    const uint32_t c = g_queue_captured.fetch_add(1, std::memory_order_relaxed);
    return c < static_cast<uint32_t>(kQueueCaptured) ? kQueueSlots - kQueueCaptured + static_cast<int>(c) : -1;
  }
  return static_cast<int>(g_queue_next.fetch_add(1, std::memory_order_relaxed) %
                          static_cast<uint64_t>(kQueueSlots - kQueueCaptured));
}
// The split kernel over ntiles tiles in mode MODE: the tile queue's
// persistent grid of min(tiles, CUs) blocks when built with it (K from the
// kernarg, K >= kQueueMinK), else one block per tile.  `share`
// (P2P_HINT_SHARE_CUS): a kernel on another stream is to run beside this one
// -- RCCL's all-gather (36.8 KiB of LDS, 8 waves of 256 VGPRs) fits no CU
// that holds a 128-KiB split block -- so one block per tile: every tile's end
// frees a CU the dispatcher can hand to it, where the persistent grid holds
// every CU until the launch ends.
template <int MODE>
static void launch_split(const float* const* peers, int K, const int32_t* k_dev, int64_t ntiles, float* w,
                         float* out, float lr, const p2p_split_tile_t* tiles, const Seg* segs,
                         const p2p_row_chunk_t* chunks, bool recip, hipStream_t st, bool share = false) {
  const dim3 block(64 * (kSL + kSC));
  const int q = use_queue<MODE>(share, k_dev, K) ? queue_slot(st) : -1;
  if (q >= 0) {
    const dim3 grid(static_cast<unsigned>(ntiles < device_cus() ? ntiles : device_cus()));
    if (recip)
      hipLaunchKernelGGL((fedavg_split_kernel<true, MODE, true>), grid, block, 0, st, peers, K, k_dev, ntiles, w, out,
                         lr, tiles, segs, chunks, q);
    else
      hipLaunchKernelGGL((fedavg_split_kernel<false, MODE, true>), grid, block, 0, st, peers, K, k_dev, ntiles, w,
                         out, lr, tiles, segs, chunks, q);
    return;
  }
  const dim3 grid = split_grid(ntiles);
  if (recip)
    hipLaunchKernelGGL((fedavg_split_kernel<true, MODE, false>), grid, block, 0, st, peers, K, k_dev, ntiles, w, out,
                       lr, tiles, segs, chunks, -1);
  else
    hipLaunchKernelGGL((fedavg_split_kernel<false, MODE, false>), grid, block, 0, st, peers, K, k_dev, ntiles, w, out,
                       lr, tiles, segs, chunks, -1);
}

static void launch_flat(const float* const* peers, int K, const int32_t* k_dev, int64_t n, float* w, float* out,
                        float lr, hipStream_t stream, bool recip = false, bool share = false) {
  int64_t done = 0;
  {
    const int64_t tiles = split_tiles_for(K, n / kSTile, use_queue<kFlat>(share, k_dev, K) && K <= kAllTilesMaxK);
    if (tiles > 0) {
      launch_split<kFlat>(peers, K, k_dev, tiles, w, out, lr, nullptr, nullptr, nullptr, recip, stream, share);
      done = tiles * kSTile;
      if (done == n) return;
    }
  }
  static_assert(kSTile % kTile == 0, "split tiles are whole VGPR tiles");
  // A remainder (or a whole buffer) of fewer 4096-float tiles than CUs --
  // the split kernel's rest: ~231 per cfg3 plane -- runs 1024-float tiles,
  // four times the blocks, so every CU streams.
#ifndef P2P_FLAT_QUARTERS
#define P2P_FLAT_QUARTERS 1
#endif
  if (P2P_FLAT_QUARTERS && ceil_div(n - done, kTile) < device_cus()) {
    const int64_t qbase = done / tile_of<1>();
    const dim3 qgrid(grid_for_tiles(ceil_div(n - done, tile_of<1>())));
    if (recip)
      hipLaunchKernelGGL((fedavg_flat_kernel<1, true>), qgrid, dim3(kBlock), 0, stream, peers, K, k_dev, n, w, out, lr,
                         qbase);
    else
      hipLaunchKernelGGL((fedavg_flat_kernel<1, false>), qgrid, dim3(kBlock), 0, stream, peers, K, k_dev, n, w, out,
                         lr, qbase);
    return;
  }
  const int64_t tile_base = done / kTile;
  const dim3 grid(grid_for_tiles(ceil_div(n - done, kTile)));
  if (recip)
    hipLaunchKernelGGL((fedavg_flat_kernel<kNV, true>), grid, dim3(kBlock), 0, stream, peers, K, k_dev, n, w, out, lr,
                       tile_base);
  else
    hipLaunchKernelGGL((fedavg_flat_kernel<kNV, false>), grid, dim3(kBlock), 0, stream, peers, K, k_dev, n, w, out,
                       lr, tile_base);
}

static int grid_stride_blocks(int64_t nblocks) {
  const int64_t cap = 256 * 8;  // 256 CUs x 8 resident blocks; grid-stride beyond
  return static_cast<int>(nblocks < cap ? (nblocks > 0 ? nblocks : 1) : cap);
}

}  // namespace p2p

using namespace p2p;

static int32_t launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? P2P_OK : static_cast<int32_t>(e);
}

extern "C" P2P_INTERNAL int64_t p2p_fedavg_tile_elems(void) { return kTile; }

static_assert(kSTile == P2P_SPLIT_TILE, "the ABI's split tile");
static_assert(kSRpw * 256 == P2P_ROW_CHUNK && kSC * P2P_ROW_CHUNK == kSTile, "a consumer wave's chunk");

extern "C" int64_t p2p_fedavg_split_plan(int32_t k, int64_t full_tiles) { return split_tiles_for(k, full_tiles); }

extern "C" int32_t p2p_fedavg_split_rows_f32(const float* const* rows, int32_t k, int64_t ntiles,
                                            const p2p_row_chunk_t* chunks, int32_t rule, float lr,
                                            p2p_stream_t stream) {
  if (!rows || !chunks || k < 1 || ntiles < 1) return P2P_ERR_INVALID;
  if (rule != P2P_RULE_FEDAVG && rule != P2P_RULE_FEDAVG_TORCH_GPU) return P2P_ERR_INVALID;
  launch_split<kRows>(rows, k, nullptr, ntiles, nullptr, nullptr, lr, nullptr, nullptr, chunks,
                      rule == P2P_RULE_FEDAVG_TORCH_GPU, static_cast<hipStream_t>(stream));
  return launch_status();
}

extern "C" int32_t p2p_fedavg_split_segments_f32(const p2p_split_tile_t* tiles, int64_t ntiles,
                                                 const p2p_segment_t* segs, int32_t k, int32_t rule, float lr,
                                                 p2p_stream_t stream) {
  if (!tiles || !segs || k < 1 || ntiles < 0) return P2P_ERR_INVALID;
  if (rule != P2P_RULE_FEDAVG && rule != P2P_RULE_FEDAVG_TORCH_GPU) return P2P_ERR_INVALID;
  if (ntiles == 0) return P2P_OK;
  launch_split<kSegs>(nullptr, k, nullptr, ntiles, nullptr, nullptr, lr, tiles, segs, nullptr,
                      rule == P2P_RULE_FEDAVG_TORCH_GPU, static_cast<hipStream_t>(stream));
  return launch_status();
}

extern "C" int32_t p2p_fedavg_split_chunks_f32(const p2p_split_tile_t* chunks, int64_t ntiles,
                                               const p2p_segment_t* segs, int32_t k, int32_t rule, float lr,
                                               p2p_stream_t stream) {
  if (!chunks || !segs || k < 1 || ntiles < 0) return P2P_ERR_INVALID;
  if (rule != P2P_RULE_FEDAVG && rule != P2P_RULE_FEDAVG_TORCH_GPU) return P2P_ERR_INVALID;
  if (ntiles == 0) return P2P_OK;
  launch_split<kChunks>(nullptr, k, nullptr, ntiles, nullptr, nullptr, lr, chunks, segs, nullptr,
                        rule == P2P_RULE_FEDAVG_TORCH_GPU, static_cast<hipStream_t>(stream));
  return launch_status();
}

P2P_INTERNAL int32_t p2p_fedavg_flat_launch(const float* const* peers, int32_t k, int64_t n, float* w,
                                            float* out, float lr, p2p_stream_t stream, int32_t recip,
                                            int32_t hints) {
  launch_flat(peers, k, nullptr, n, w, out, lr, static_cast<hipStream_t>(stream), recip != 0,
              (hints & P2P_HINT_SHARE_CUS) != 0);
  return launch_status();
}

extern "C" int32_t p2p_fedavg_apply_f32(const float* const* peers, int32_t k, int64_t n, float* w,
                                        float lr, p2p_stream_t stream) {
  if (!peers || !w || k < 1 || n < 0) return P2P_ERR_INVALID;
  if (reinterpret_cast<uintptr_t>(w) & 3) return P2P_ERR_ALIGN;
  if (n == 0) return P2P_OK;
  launch_flat(peers, k, nullptr, n, w, nullptr, lr, static_cast<hipStream_t>(stream));
  return launch_status();
}

extern "C" int32_t p2p_mean_f32(const float* const* peers, int32_t k, int64_t n, float* out,
                                p2p_stream_t stream) {
  if (!peers || !out || k < 1 || n < 0) return P2P_ERR_INVALID;
  if (reinterpret_cast<uintptr_t>(out) & 3) return P2P_ERR_ALIGN;
  if (n == 0) return P2P_OK;
  launch_flat(peers, k, nullptr, n, nullptr, out, 0.f, static_cast<hipStream_t>(stream));
  return launch_status();
}

extern "C" int32_t p2p_fedavg_apply_devk_f32(const float* const* peers, const int32_t* k_dev,
                                             int32_t k_max, int64_t n, float* w, float lr,
                                             float* out, p2p_stream_t stream) {
  if (!peers || !k_dev || (!w && !out) || k_max < 1 || n < 0) return P2P_ERR_INVALID;
  if ((reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(out)) & 3) return P2P_ERR_ALIGN;
  if (n == 0) return P2P_OK;
  launch_flat(peers, k_max, k_dev, n, w, out, lr, static_cast<hipStream_t>(stream));
  return launch_status();
}

extern "C" P2P_INTERNAL int32_t p2p_fedavg_segments_f32(const p2p_segment_t* segs, int32_t nseg,
                                           int64_t total_tiles, int32_t k, float lr,
                                           p2p_stream_t stream, int32_t recip) {
  if (!segs || nseg < 1 || k < 1 || total_tiles < 0) return P2P_ERR_INVALID;
  if (total_tiles == 0) return P2P_OK;
  static_assert(kTile == 4 * tile_of<1>(), "four quarters per tile");
  const hipStream_t st = static_cast<hipStream_t>(stream);
  if (total_tiles < device_cus()) {
    const dim3 grid(static_cast<unsigned>(4 * total_tiles));
    if (recip) hipLaunchKernelGGL((fedavg_segments_kernel<true, true>), grid, dim3(kBlock), 0, st, segs, nseg, k, lr);
    else hipLaunchKernelGGL((fedavg_segments_kernel<false, true>), grid, dim3(kBlock), 0, st, segs, nseg, k, lr);
    return launch_status();
  }
  const dim3 grid(static_cast<unsigned>(total_tiles));
  if (recip) hipLaunchKernelGGL(fedavg_segments_kernel<true>, grid, dim3(kBlock), 0, st, segs, nseg, k, lr);
  else hipLaunchKernelGGL(fedavg_segments_kernel<false>, grid, dim3(kBlock), 0, st, segs, nseg, k, lr);
  return launch_status();
}

extern "C" int32_t p2p_apply_f32(float* w, const float* agg, float lr, int64_t n,
                                 p2p_stream_t stream) {
  if (!w || !agg || n < 0) return P2P_ERR_INVALID;
  if ((reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(agg)) & 3) return P2P_ERR_ALIGN;
  if (n == 0) return P2P_OK;
  hipLaunchKernelGGL(apply_kernel, dim3(grid_stride_blocks(ceil_div(n, kBlock * 4))), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), w, agg, lr, n);
  return launch_status();
}
