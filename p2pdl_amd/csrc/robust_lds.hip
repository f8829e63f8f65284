// K2 (K in 65..256) -- coordinate-wise median / trimmed mean with L lanes
// per coordinate and the peer rows staged HBM -> LDS by LDS-DMA.
//
// Rule (no reference implementation, README.md:10):
//   median : key of rank (K-1)/2 under the IEEE total order on float bits
//   trimmed: b = floor(0.2 K); fp32 sum of ranks b..K-b-1 ascending from +0,
//            IEEE-divided by K-2b
// then w += lr*agg, multiply and add separately rounded (aggregation.py:36-38).
//
// Layout.  A block's 4 sorter waves own a tile of 256/L coordinates; wave wi
// takes coordinates [wi*64/L, (wi+1)*64/L) and lane = L*c + q holds
// keys q*H .. q*H+H-1 (H = KP/L) of coordinate c, so every cross-lane step
// is a DPP quad_perm inside a quad, never LDS.  Each lane sorts its H keys
// in VGPRs (Batcher network), then the L slices are merged bitonically:
// stage s (2, 4 lanes) = a FLIP against lane q^(s-1) (register j vs the
// partner's H-1-j), half-cleaners against q^d, and an in-register bitonic
// merge.  A keep-min / keep-max against the partner is ONE v_med3_u32 with a
// lane-constant 0 / ~0 third operand (plus the DPP move).
//
// Staging.  The block's LDS image holds its tile as L slices of H rows x 64
// floats (row = one peer, 256 contiguous bytes in HBM) plus the w row.  The
// next tile's rows are requested with global_load_lds_dwordx4 (1 KiB = 4
// rows per wave-instruction, no VGPR destination, the L waves split the
// pieces) as soon as the current tile has been read into registers, so the
// HBM latency hides behind the sort and the register file holds one tile.
// Two barriers per tile: after the DMA lands (vmcnt(0) + s_barrier) and after
// the image is read (lgkmcnt(0) + s_barrier) before it is overwritten.
// Slices are padded by 128/L bytes so the L lanes of a coordinate hit
// different banks.  Measured: per-wave tiles with 64-B rows (16 coordinates)
// ran 34% of HBM peak at K = 256 -- 256-B rows per peer are what the HBM
// side needs (FedAvg reads 1 KiB runs).
//
// XCD placement: logical block g = (blockIdx % 8) * (grid / 8) + blockIdx / 8,
// so neighbouring tiles are read through the same XCD's L2.
//
// Tiles that cannot be DMA'd (a peer / w pointer not 16-B aligned, or the
// ragged last tile of a buffer) load the same keys with per-lane global
// loads; the arithmetic after the load is the same code.
#include "robust_nets.h"

#define P2P_LDS __attribute__((address_space(3)))

namespace p2p {


// DPP move with bound_ctrl: every lane is written, so no "old" operand has to
// be materialised (update_dpp(0, ...) cost a v_mov_b32 per exchange).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t x) {
  return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(x), CTRL, 0xF, 0xF, true));
}
// value of lane (lane ^ M) inside the quad
template <int M>
__device__ __forceinline__ uint32_t xq(uint32_t x) {
  static_assert(M >= 1 && M <= 3, "quad partner");
  return dpp<M == 1 ? 0xB1 : (M == 2 ? 0x4E : 0x1B)>(x);
}
template <int M>
__device__ __forceinline__ fk xq(fk x) {
  return fk{__uint_as_float(xq<M>(__float_as_uint(x.x)))};
}

// Type-generic pieces of the L-lane reduction: uint32 total-order keys or
// float values (NaN-free waves, robust_nets.h; keep / keep_limit there);
// value() is the float the element stands for.
__device__ __forceinline__ float value(uint32_t k) { return __uint_as_float(key2f(k)); }
__device__ __forceinline__ float value(fk f) { return f.x; }

// value of slice q-1 of the same coordinate (slice 0 receives its own)
template <int L>
__device__ __forceinline__ float from_prev_slice(float x) {
  static_assert(L == 2 || L == 4, "lanes per coordinate");
  return __uint_as_float(dpp<L == 4 ? 0x90 : 0xA0>(__float_as_uint(x)));
}

template <int L, int H, int NB = 0>
struct LdsLayout {
  static constexpr int W = 4;                  // sorter waves per block (and as many loaders)
  static constexpr int TB = 64 * W / L;        // coordinates per block tile
  static constexpr int TW = 64 / L;            // coordinates per sorter wave
  static constexpr int RB = 4 * TB;            // bytes per peer row (>= 256 contiguous in HBM)
  static constexpr int PAD = L > 1 ? 128 / L : 0;
  static constexpr int SB = H * RB + PAD;      // bytes per slice
  static constexpr int WOFF = L * SB;          // w row
  static constexpr int IMG = (WOFF + RB + 15) / 16 * 16;  // one tile image
  static constexpr int NBUF = NB ? NB : (2 * IMG <= 160 * 1024 ? 2 : 1);  // images (tiles in flight)
  static constexpr int BYTES = NBUF * IMG;
  static constexpr int RPP = 1024 / RB;        // peer rows per 1 KiB DMA piece
  static constexpr int LPR = RB / 16;          // lanes per row of a piece
  static constexpr int CPS = H * RB / 1024;    // pieces per slice
  static constexpr int NCHW = CPS * L / W;     // pieces per loader wave per tile
  static_assert(RB <= 1024 && (H * RB) % 1024 == 0 && NCHW * W == CPS * L, "whole 1 KiB DMA pieces");
  static_assert(BYTES <= 160 * 1024, "LDS");
};

__device__ __forceinline__ void glds16(const float* src, uint8_t P2P_LDS* dst) {
  __builtin_amdgcn_global_load_lds((P2P_GLOBAL void*)(const_cast<float*>(src)), (P2P_LDS void*)dst, 16, 0, 0);
}

// Where a tile lives (flat buffer or one segment of a state_dict).
struct TileSrc {
  const float* const* peers;
  float* w;
  float* out;
  int64_t n;
  int64_t c0;   // first coordinate of the tile inside the buffer
  int64_t seg;  // identity of the source (its first tile) for the pointer cache
};

template <int TW, bool SEGS>
__device__ __forceinline__ TileSrc locate(const float* const* peers, const Seg* segs, int nseg, int64_t n,
                                          float* w, float* out, int64_t t) {
  if constexpr (SEGS) {
    const Seg s = load_segment(segs, nseg, t);
    return TileSrc{s.peers, s.w, s.out, s.n, (t - s.tile_begin) * TW, s.tile_begin};
  } else {
    return TileSrc{peers, w, out, n, t * TW, 0};
  }
}

// The L-lane reduction of one coordinate.  v[] holds this lane's H elements
// (uint32 keys, pads 0xFFFFFFFF; or float values, pads +inf); returns the
// aggregate, valid in the lane where `own` is set on return.
template <int L, int H, int RULE, int MODE, typename T>
__device__ __forceinline__ float reduce_keys(T (&v)[H], int q, int K, int trim_b, bool& own) {
  static_assert(L == 1 || L == 2 || L == 4, "lanes per coordinate");
  if constexpr (L == 1) {
    if constexpr (MODE == 0) sort_full<H>(v); else run_special<H, MODE>(v);
    own = true;
    if constexpr (RULE == P2P_RULE_MEDIAN) {
      if constexpr (MODE == 1) return value(v[(H - 1) / 2]);
      const int r = (K - 1) / 2;
      T sel = v[0];
#pragma unroll
      for (int j = 1; j < H; ++j) sel = (j == r) ? v[j] : sel;
      return value(sel);
    } else {
      float acc = 0.f;
      if constexpr (MODE == 2) {
        constexpr int b = (H * 2) / 10;
#pragma unroll
        for (int j = b; j < H - b; ++j) acc = __fadd_rn(acc, value(v[j]));
        return acc / static_cast<float>(H - 2 * b);
      }
      const int hi = K - trim_b;
#pragma unroll
      for (int j = 0; j < H; ++j)
        if (j >= trim_b && j < hi) acc = __fadd_rn(acc, value(v[j]));  // uniform predicate
      return acc / static_cast<float>(K - 2 * trim_b);
    }
  } else {
    sort_full<H>(v);
#pragma unroll
    for (int s = 2; s <= L; s *= 2) {
      if constexpr (RULE == P2P_RULE_MEDIAN && MODE == 1) {
        if (s == L) {  // last flip: slices q < L/2 keep the K/2 smallest; the median is their max.
          // Only those lanes' results are used, so each pair is ONE v_min with
          // the partner's register as a DPP operand (no v_mov_dpp, no med3),
          // reduced by v_max3.
          T mx = min(v[0], L == 2 ? xq<1>(v[H - 1]) : xq<3>(v[H - 1]));
#pragma unroll
          for (int j = 1; j < H; ++j) mx = max(mx, min(v[j], L == 2 ? xq<1>(v[H - 1 - j]) : xq<3>(v[H - 1 - j])));
          if constexpr (L == 4) mx = max(mx, xq<1>(mx));
          own = (q == 0);
          return value(mx);
        }
      }
      {  // flip against the mirrored lane of the s-lane group
        const T lim = keep_limit(v[0], (q & (s / 2)) != 0);
#pragma unroll
        for (int j = 0; j < H / 2; ++j) {
          const T a = v[j], b = v[H - 1 - j];
          const T pa = (s == 2) ? xq<1>(b) : xq<3>(b);  // partner's v[H-1-j]
          const T pb = (s == 2) ? xq<1>(a) : xq<3>(a);  // partner's v[j]
          v[j] = keep(a, pa, lim);
          v[H - 1 - j] = keep(b, pb, lim);
        }
      }
#pragma unroll
      for (int d = s / 4; d >= 1; d /= 2) {  // half-cleaners (only at s = 4: d = 1)
        const T lim = keep_limit(v[0], (q & d) != 0);
#pragma unroll
        for (int j = 0; j < H; ++j) v[j] = keep(v[j], xq<1>(v[j]), lim);
      }
      bmerge<H>(v);
    }
    // slice q now holds ranks q*H .. q*H+H-1, ascending
    if constexpr (RULE == P2P_RULE_MEDIAN) {
      const int r = (K - 1) / 2;
      const int rl = r % H;
      T sel = v[0];
#pragma unroll
      for (int j = 1; j < H; ++j) sel = (j == rl) ? v[j] : sel;
      own = (q == r / H);
      return value(sel);
    } else {
      // ascending-rank sequential sum from +0: slice 0's ranks, then slice 1 ...
      constexpr int KP = L * H;
      const int b = MODE == 2 ? (KP * 2) / 10 : trim_b;
      const int hi = MODE == 2 ? KP - b : K - trim_b;
      float f[H];
#pragma unroll
      for (int j = 0; j < H; ++j) f[j] = value(v[j]);  // once: a value is summed in up to L phases
      float acc = 0.f;
#pragma unroll
      for (int p = 0; p < L; ++p) {
        float a = p == 0 ? 0.f : from_prev_slice<L>(acc);
#pragma unroll
        for (int j = 0; j < H; ++j) {
          const int g = p * H + j;
          if (g >= b && g < hi)  // wave-uniform
            a = __fadd_rn(a, f[j]);
        }
        acc = (q == p) ? a : acc;
      }
      own = (q == L - 1);
      return acc / static_cast<float>(MODE == 2 ? KP - 2 * b : K - 2 * trim_b);
    }
  }
}

// Register-staged fill of the LDS image for a tile that cannot be DMA'd
// (misaligned pointer or ragged tail): each lane writes exactly the words it
// reads back.  Out of line: its row-pointer loads must not share the
// register budget of the sorting loop.
template <int L, int H>
__device__ __attribute__((noinline)) void fill_direct(uint8_t P2P_LDS* lds, const float* const* tbl,
                                                      const float* w, int64_t n, int64_t i, int K, int q,
                                                      int c) {
  using Lay = LdsLayout<L, H>;
  const int64_t ic = i < n ? i : n - 1;  // dead lanes re-read the last element
  uint32_t P2P_LDS* sl = (uint32_t P2P_LDS*)(lds + q * Lay::SB) + c;
#pragma unroll
  for (int j0 = 0; j0 < H; j0 += 16) {
    uint32_t x[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int row = q * H + j0 + j;
      x[j] = __float_as_uint(ldg(table_at(tbl, row < K ? row : K - 1) + ic));
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) sl[(j0 + j) * (Lay::RB / 4)] = x[j];
  }
  if (w && q == 0) ((float P2P_LDS*)(lds + Lay::WOFF))[c] = ldg(w + ic);
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (immediate operand).
template <int N = 0>
__device__ __forceinline__ void wait_vmcnt(int n) {
  if constexpr (N > 24) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (n == N) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
    else wait_vmcnt<N + 1>(n);
  }
}

// Block barrier once this wave's vector-memory ops older than the `younger`
// most recent ones have completed (the DMA of the tile about to be read).
__device__ __forceinline__ void block_sync_vm(int younger) {
  wait_vmcnt(younger);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void block_sync_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Block = 4 sorter waves + 4 loader waves.  Loaders only issue the LDS-DMA
// (a global_load_lds costs its wave ~100 cycles of issue; the sorters' VALU
// stream never pays it); sorters read the image, sort, store.  The block
// walks tiles t, t+grid, ... with two images: loaders keep the DMA of the
// next tile in flight while the sorters work on the current one.  Per tile:
//   loaders: wait own pieces of tile t | barrier A | barrier B | DMA(t+2 grid)
//   sorters: (fill if not DMA-able)   | barrier A | read      | barrier B | sort, store
template <int L, int H, int RULE, int MODE, bool SEGS, int NB>
__global__ __launch_bounds__(512) void robust_lds_kernel(const float* const* __restrict__ peers,
                                                             const Seg* __restrict__ segs, int nseg,
                                                             int64_t ntiles, int K, int trim_b, int64_t n,
                                                             float* w, float* out, float lr, int64_t nb) {
  using Lay = LdsLayout<L, H, NB>;
  static_assert(128 * Lay::W == 512, "launch bounds");
  __shared__ __attribute__((aligned(16))) uint8_t lds_raw[Lay::BYTES];
  uint8_t P2P_LDS* lds = (uint8_t P2P_LDS*)lds_raw;
  const int wi = __builtin_amdgcn_readfirstlane(static_cast<int>(tid_x() >> 6));
  const int lane = tid_x() & 63;
  const bool loader = wi >= Lay::W;  // wave-uniform role
  const int li = wi - Lay::W;        // loader index
  const int q = lane % L, c = wi * Lay::TW + lane / L;  // sorters: coordinate inside the block tile

  // nb: the grid size, passed by the launch (the persistent loop strides by it)
  int64_t t = bid_x();
  if ((nb & 7) == 0) t = (bid_x() & 7) * (nb >> 3) + (bid_x() >> 3);  // XCD-contiguous tiles
  if (t >= ntiles) return;

  // loaders: per-lane row pointers of their DMA pieces for the bound source.
  // Cached in VGPRs when two images are in flight (the loader must not wait
  // on a pointer load while the next tile's DMA is outstanding); with one
  // image they are reloaded per tile (L2 hits) so the sorters' 128 keys keep
  // the register file.
  constexpr bool kCachePtr = Lay::NBUF == 2;
  const float* rp[kCachePtr ? Lay::NCHW : 1];
  int64_t cur_seg = -1;
  bool aligned = false;
  auto row_of = [&](int m) {
    const int ch = li * Lay::NCHW + m;
    const int row = (ch / Lay::CPS) * H + (ch % Lay::CPS) * Lay::RPP + lane / Lay::LPR;
    return row < K ? row : K - 1;
  };
  auto bind = [&](const TileSrc& s) {
    if (s.seg == cur_seg) return;
    cur_seg = s.seg;
    aligned = all_aligned16(s.peers, K, s.w, nullptr);
    if constexpr (kCachePtr) {
      if (loader) {
#pragma unroll
        for (int m = 0; m < Lay::NCHW; ++m) rp[m] = table_at(s.peers, row_of(m));
      }
    }
  };
  auto dma_ok = [&](const TileSrc& s) { return aligned && s.c0 + Lay::TB <= s.n; };
  auto real_piece = [&](int m) {  // pieces made only of pad rows are skipped (MODE 0)
    const int ch = li * Lay::NCHW + m;
    return MODE != 0 || (ch / Lay::CPS) * H + (ch % Lay::CPS) * Lay::RPP < K;
  };
  auto npieces = [&](const TileSrc& s) {
    int np = 0;
#pragma unroll
    for (int m = 0; m < Lay::NCHW; ++m) np += real_piece(m) ? 1 : 0;
    return np + ((s.w && li == 0) ? 1 : 0);
  };
  auto issue = [&](const TileSrc& s, int img_off) {
    uint8_t P2P_LDS* im = lds + img_off;
    const int64_t off = s.c0 + 4 * (lane % Lay::LPR);
#pragma unroll
    for (int m = 0; m < Lay::NCHW; ++m) {
      const int ch = li * Lay::NCHW + m;
      if (real_piece(m)) {
        const float* src = kCachePtr ? rp[kCachePtr ? m : 0] : table_at(s.peers, row_of(m));
        glds16(src + off, im + (ch / Lay::CPS) * Lay::SB + (ch % Lay::CPS) * 1024);
      }
    }
    if (s.w && li == 0 && lane < Lay::LPR) glds16(s.w + s.c0 + 4 * lane, im + Lay::WOFF);
  };

  // NBUF images: tile t in image `img` while the DMA of the next NBUF-1 tiles
  // fills the others; the DMA of tile t + NBUF*grid goes into `img` as soon
  // as tile t has been read into registers.  Loaders and sorters run separate
  // loops (same tile sequence, same two barriers per tile) so neither role's
  // registers are live across the other's code.
  constexpr int D = Lay::NBUF;
  TileSrc cur = locate<Lay::TB, SEGS>(peers, segs, nseg, n, w, out, t);
  bind(cur);
  bool dma_cur = dma_ok(cur);
  if (loader && dma_cur) issue(cur, 0);
  TileSrc nx1 = cur;
  bool dma_nx1 = false;
  if (D == 2 && t + nb < ntiles) {
    nx1 = locate<Lay::TB, SEGS>(peers, segs, nseg, n, w, out, t + nb);
    bind(nx1);
    dma_nx1 = dma_ok(nx1);
    if (loader && dma_nx1) issue(nx1, Lay::IMG);
  }
  int img = 0;
  // the tile D grids ahead of t: located, and DMA'd by the loaders
  auto advance = [&](int64_t tt) {
    TileSrc nxd = D == 2 ? nx1 : cur;
    bool dma_nxd = false;
    if (tt + D * nb < ntiles) {
      nxd = locate<Lay::TB, SEGS>(peers, segs, nseg, n, w, out, tt + D * nb);
      bind(nxd);
      dma_nxd = dma_ok(nxd);
      if (loader && dma_nxd) issue(nxd, img);
    }
    if constexpr (D == 2) {
      cur = nx1;
      dma_cur = dma_nx1;
      nx1 = nxd;
      dma_nx1 = dma_nxd;
      img ^= Lay::IMG;
    } else {
      cur = nxd;
      dma_cur = dma_nxd;
    }
  };

  if (loader) {
    for (; t < ntiles; t += nb) {
      block_sync_vm(D == 2 && dma_nx1 ? npieces(nx1) : 0);  // A: this loader's pieces of tile t landed
      __builtin_amdgcn_s_barrier();                         // B: sorters have read the image
      asm volatile("" ::: "memory");
      advance(t);
    }
    return;
  }
  for (; t < ntiles; t += nb) {
    uint8_t P2P_LDS* im = lds + img;
    const TileSrc me = cur;
    const int64_t i = me.c0 + c;
    if (!dma_cur) fill_direct<L, H>(im, me.peers, me.w, me.n, i, K, q, c);
    __builtin_amdgcn_s_barrier();  // A: every piece of tile t is in the image
    asm volatile("" ::: "memory");
    uint32_t v[H];
    const uint32_t P2P_LDS* sl = (const uint32_t P2P_LDS*)(im + q * Lay::SB) + c;
#pragma unroll
    for (int j = 0; j < H; ++j) v[j] = sl[j * (Lay::RB / 4)];
    const float wv = me.w ? ((const float P2P_LDS*)(im + Lay::WOFF))[c] : 0.f;
    block_sync_lds();  // B: image consumed, free for the DMA D tiles ahead
    advance(t);
    bool own = false;
    float agg;
    bool fast = false;  // every slot real (K == KP) and no NaN in the wave: the float network
    if constexpr (MODE != 0) fast = !wave_has_nan(v);
    if (fast) {
      fk f[H];
#pragma unroll
      for (int j = 0; j < H; ++j) f[j].x = __uint_as_float(v[j]);
      agg = reduce_keys<L, H, RULE, MODE>(f, q, K, trim_b, own);
    } else {
#pragma unroll
      for (int j = 0; j < H; ++j) {
        const bool real = (MODE != 0) || (q * H + j < K);
        v[j] = real ? f2key(v[j]) : 0xFFFFFFFFu;  // pads sort after every real key
      }
      agg = reduce_keys<L, H, RULE, MODE>(v, q, K, trim_b, own);
    }
    if (own && i < me.n) {
      if (me.out) stg(me.out + i, agg);
      if (me.w) stg(me.w + i, apply_lr(wv, lr, agg));
    }
  }
}

// Two sorter groups per block (lab variant 7): 2 x 4 sorter waves + 4 loader
// waves = 12 waves, 3 per SIMD, so every SIMD has TWO sorting waves to issue
// from (a lone sorter wave leaves ~11% of its cycles idle on LDS latency and
// barriers).  Group g sorts the tiles of image g: iteration i covers tiles
// t + 2i*grid (image 0) and t + (2i+1)*grid (image 1); the loaders refill both
// images as soon as both groups have read them (one DMA period of slack, not
// two).  768-lane blocks cap the kernel at 168 VGPRs: uint32-key network only.
template <int RULE, int MODE, bool SEGS>
__global__ __launch_bounds__(768) void robust_lds_g2_kernel(const float* const* __restrict__ peers,
                                                            const Seg* __restrict__ segs, int nseg,
                                                            int64_t ntiles, int K, int trim_b, int64_t n,
                                                            float* w, float* out, float lr, int64_t nb) {
  constexpr int L = 4, H = 64;
  using Lay = LdsLayout<L, H>;
  static_assert(Lay::NBUF == 2 && Lay::W == 4, "one image per sorter group");
  __shared__ __attribute__((aligned(16))) uint8_t lds_raw[Lay::BYTES];
  uint8_t P2P_LDS* lds = (uint8_t P2P_LDS*)lds_raw;
  const int wi = __builtin_amdgcn_readfirstlane(static_cast<int>(tid_x() >> 6));
  const int lane = tid_x() & 63;
  const bool loader = wi >= 2 * Lay::W;  // wave-uniform role
  const int g = loader ? 0 : wi / Lay::W;
  const int li = wi - 2 * Lay::W;
  const int q = lane % L, c = (wi % Lay::W) * Lay::TW + lane / L;

  // nb: the grid size, passed by the launch (the persistent loop strides by it)
  int64_t t0 = bid_x();
  if ((nb & 7) == 0) t0 = (bid_x() & 7) * (nb >> 3) + (bid_x() >> 3);  // XCD-contiguous tiles
  if (t0 >= ntiles) return;  // block-uniform
  const int64_t iters = ceil_div(ceil_div(ntiles - t0, nb), 2);
  auto tile_at = [&](int64_t i, int gg) { return t0 + (2 * i + gg) * nb; };

  const float* rp[Lay::NCHW];
  int64_t cur_seg = -1;
  bool aligned = false;
  auto row_of = [&](int m) {
    const int ch = li * Lay::NCHW + m;
    const int row = (ch / Lay::CPS) * H + (ch % Lay::CPS) * Lay::RPP + lane / Lay::LPR;
    return row < K ? row : K - 1;
  };
  auto bind = [&](const TileSrc& s) {
    if (s.seg == cur_seg) return;
    cur_seg = s.seg;
    aligned = all_aligned16(s.peers, K, s.w, nullptr);
    if (loader) {
#pragma unroll
      for (int m = 0; m < Lay::NCHW; ++m) rp[m] = table_at(s.peers, row_of(m));
    }
  };
  auto dma_ok = [&](const TileSrc& s) { return aligned && s.c0 + Lay::TB <= s.n; };
  auto real_piece = [&](int m) {
    const int ch = li * Lay::NCHW + m;
    return MODE != 0 || (ch / Lay::CPS) * H + (ch % Lay::CPS) * Lay::RPP < K;
  };
  auto issue = [&](const TileSrc& s, int img_off) {
    uint8_t P2P_LDS* im = lds + img_off;
    const int64_t off = s.c0 + 4 * (lane % Lay::LPR);
#pragma unroll
    for (int m = 0; m < Lay::NCHW; ++m) {
      const int ch = li * Lay::NCHW + m;
      if (real_piece(m)) glds16(rp[m] + off, im + (ch / Lay::CPS) * Lay::SB + (ch % Lay::CPS) * 1024);
    }
    if (s.w && li == 0 && lane < Lay::LPR) glds16(s.w + s.c0 + 4 * lane, im + Lay::WOFF);
  };
  auto stage = [&](int64_t i) {  // loaders: DMA of iteration i's tiles into images 0 and 1
#pragma unroll
    for (int gg = 0; gg < 2; ++gg) {
      const int64_t tt = tile_at(i, gg);
      if (tt < ntiles) {
        const TileSrc s = locate<Lay::TB, SEGS>(peers, segs, nseg, n, w, out, tt);
        bind(s);
        if (dma_ok(s)) issue(s, gg * Lay::IMG);
      }
    }
  };

  if (loader) {
    stage(0);
    for (int64_t i = 0; i < iters; ++i) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this loader's pieces of iteration i landed
      __builtin_amdgcn_s_barrier();                     // A
      __builtin_amdgcn_s_barrier();                     // B: both groups have read their image
      asm volatile("" ::: "memory");
      stage(i + 1);
    }
    return;
  }
  uint8_t P2P_LDS* im = lds + g * Lay::IMG;
  for (int64_t i = 0; i < iters; ++i) {
    const int64_t tt = tile_at(i, g);
    const bool has = tt < ntiles;  // the last iteration may hold one tile only
    TileSrc me{};
    if (has) {
      me = locate<Lay::TB, SEGS>(peers, segs, nseg, n, w, out, tt);
      bind(me);
      if (!dma_ok(me)) fill_direct<L, H>(im, me.peers, me.w, me.n, me.c0 + c, K, q, c);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // A: both images hold their tiles
    asm volatile("" ::: "memory");
    uint32_t v[H];
    const uint32_t P2P_LDS* sl = (const uint32_t P2P_LDS*)(im + q * Lay::SB) + c;
#pragma unroll
    for (int j = 0; j < H; ++j) v[j] = sl[j * (Lay::RB / 4)];
    const float wv = (has && me.w) ? ((const float P2P_LDS*)(im + Lay::WOFF))[c] : 0.f;
    block_sync_lds();  // B: images consumed
    if (!has) continue;
#pragma unroll
    for (int j = 0; j < H; ++j) {
      const bool real = (MODE != 0) || (q * H + j < K);
      v[j] = real ? f2key(v[j]) : 0xFFFFFFFFu;
    }
    bool own = false;
    const float agg = reduce_keys<L, H, RULE, MODE>(v, q, K, trim_b, own);
    const int64_t e = me.c0 + c;
    if (own && e < me.n) {
      if (me.out) stg(me.out + e, agg);
      if (me.w) stg(me.w + e, apply_lr(wv, lr, agg));
    }
  }
}

struct LdsArgs {
  const float* const* peers;
  const Seg* segs;
  int nseg;
  int64_t tiles;  // SEGS: total tiles (tile_begin prefix sums use TW)
  int K, trim_b;
  int64_t n;
  float* w;
  float* out;
  float lr;
  hipStream_t stream;
};

template <int L, int H, int RULE, int MODE, bool SEGS, int NB>
static void launch_lds_kernel(const LdsArgs& a) {
  using Lay = LdsLayout<L, H, NB>;
  auto kern = robust_lds_kernel<L, H, RULE, MODE, SEGS, NB>;
  constexpr int kThreads = 128 * Lay::W;
  static int resident = 0;  // persistent grid: every resident block slot once
  if (resident == 0) {
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kern), kThreads, 0);
    resident = (cus > 0 ? cus : 256) * (per_cu > 0 ? per_cu : 1);
  }
  const int64_t ntiles = SEGS ? a.tiles : ceil_div(a.n, Lay::TB);
  const int64_t grid = ntiles < resident ? ntiles : resident;
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(grid)), dim3(kThreads), 0, a.stream, a.peers, a.segs, a.nseg,
                     ntiles, a.K, a.trim_b, a.n, a.w, a.out, a.lr, grid);
}

template <int RULE, int MODE, bool SEGS>
static void launch_lds_g2_kernel(const LdsArgs& a) {
  using Lay = LdsLayout<4, 64>;
  auto kern = robust_lds_g2_kernel<RULE, MODE, SEGS>;
  static int resident = 0;
  if (resident == 0) {
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kern), 768, 0);
    resident = (cus > 0 ? cus : 256) * (per_cu > 0 ? per_cu : 1);
  }
  const int64_t ntiles = SEGS ? a.tiles : ceil_div(a.n, Lay::TB);
  const int64_t grid = ntiles < resident ? ntiles : resident;
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(grid)), dim3(768), 0, a.stream, a.peers, a.segs, a.nseg,
                     ntiles, a.K, a.trim_b, a.n, a.w, a.out, a.lr, grid);
}

template <int RULE>
static void launch_lds_g2(const LdsArgs& a) {
  constexpr int KP = 256;
  const bool special = RULE == P2P_RULE_MEDIAN ? a.K == KP : (a.K == KP && a.trim_b == (KP * 2) / 10);
  if (special) {
    if (a.segs) launch_lds_g2_kernel<RULE, RULE == P2P_RULE_MEDIAN ? 1 : 2, true>(a);
    else launch_lds_g2_kernel<RULE, RULE == P2P_RULE_MEDIAN ? 1 : 2, false>(a);
  } else {
    if (a.segs) launch_lds_g2_kernel<RULE, 0, true>(a);
    else launch_lds_g2_kernel<RULE, 0, false>(a);
  }
}

template <int L, int H, int RULE, int MODE, int NB>
static void launch_lds_mode(const LdsArgs& a) {
  if (a.segs) launch_lds_kernel<L, H, RULE, MODE, true, NB>(a);
  else launch_lds_kernel<L, H, RULE, MODE, false, NB>(a);
}

template <int L, int H, int RULE, int NB = 0>
static void launch_lds(const LdsArgs& a) {
  constexpr int KP = L * H;
  if constexpr (RULE == P2P_RULE_MEDIAN) {
    if (a.K == KP) return launch_lds_mode<L, H, RULE, 1, NB>(a);
  } else {
    if (a.K == KP && a.trim_b == (KP * 2) / 10) return launch_lds_mode<L, H, RULE, 2, NB>(a);
  }
  launch_lds_mode<L, H, RULE, 0, NB>(a);
}

}  // namespace p2p

using namespace p2p;

// K in 129..256: 4 lanes x 64 keys per coordinate, 64-coordinate tiles in
// both block shapes (p2p_robust_lds_tile and the launch must agree; the tile
// size is a pure function of (rule, k)).  Other
// instantiations of the templates above (4 x 32, 2 x 64, 1 x 128, 2 x 128)
// are built only into the A/B library of tools/robust_lab.hip.
extern "C" P2P_INTERNAL int64_t p2p_robust_pair_tile(int32_t rule);
// K > 128: the median always runs the pair kernels (any K, padded), whose
// tile is p2p_robust_pair_tile; the trimmed mean runs them or these LDS
// kernels by the trim, on the same 64-coordinate tile.
extern "C" P2P_INTERNAL int64_t p2p_robust_lds_tile(int32_t rule, int32_t k) {
  (void)k;
  static_assert(LdsLayout<4, 64>::TB == 64, "trimmed: pair and LDS kernels share the tile");
  return rule == P2P_RULE_MEDIAN ? p2p_robust_pair_tile(rule) : LdsLayout<4, 64>::TB;
}

extern "C" P2P_INTERNAL int32_t p2p_robust_pair_fits(int32_t rule, int32_t k, int32_t trim_b);
extern "C" P2P_INTERNAL void p2p_robust_pair_launch(const float* const* peers, const p2p_segment_t* segs,
                                                    int32_t nseg, int64_t tiles, int32_t rule, int32_t k,
                                                    int32_t trim_b, int64_t n, float* w, float* out, float lr,
                                                    p2p_stream_t stream);

// K in 129..256 with the median or a trim the pads fit (every K at the
// default 0.2): one lane per coordinate in two-wave blocks, robust_pair.hip,
// the block padded to 256 (round 4; 2-3x faster than these LDS kernels at
// K = 200).  Any other trim runs the generic padded network here, where two
// sorter groups per block were faster than one (round-2 lab A/B,
// profiles/r02/ab/labg2k).
extern "C" P2P_INTERNAL void p2p_robust_lds_launch(const float* const* peers, const p2p_segment_t* segs,
                                                   int32_t nseg, int64_t tiles, int32_t k, int32_t rule,
                                                   int32_t trim_b, int64_t n, float* w, float* out, float lr,
                                                   p2p_stream_t stream) {
  LdsArgs a{peers, segs, nseg, tiles, k, trim_b, n, w, out, lr, static_cast<hipStream_t>(stream)};
  // the median fits the pair kernels at every K in 129..256 (its tile differs
  // from these kernels': p2p_robust_lds_tile)
  if (rule == P2P_RULE_MEDIAN || p2p_robust_pair_fits(rule, k, trim_b)) {
    p2p_robust_pair_launch(peers, segs, nseg, tiles, rule, k, trim_b, n, w, out, lr, stream);
  } else {
    if (segs) launch_lds_g2_kernel<P2P_RULE_TRIMMED, 0, true>(a); else launch_lds_g2_kernel<P2P_RULE_TRIMMED, 0, false>(a);
  }
}
