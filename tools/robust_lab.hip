// A/B library for the robust kernels -- NOT the product.  It compiles the
// product's robust_lds.hip and exposes the
// template instantiations the product dispatch does not use, so variants can
// be timed and bit-compared against the product kernel on the same inputs.
// Built by `make -C p2pdl_amd/csrc lab` into tools/libp2pdl_lab.so (the
// product objects minus robust_lds.o, plus this file); selected with
// P2P_LIB=tools/libp2pdl_lab.so by tools/lab_robust.py.
#include "../p2pdl_amd/csrc/robust_lds.hip"

using namespace p2p;

namespace p2p {
// Two sorter groups per block, ASYNCHRONOUS (lab variant 8): the same 12
// waves and one image per group as robust_lds_g2_kernel, but no block
// barriers -- per-image LDS counters instead: `full[g]` (+1 per loader once
// its DMA pieces of the image's tile landed) and `empty[g]` (+1 per sorter
// wave once it has read the image).  Tile j of the block goes to image /
// group j & 1; a loader refills image j & 1 with tile j + 2 as soon as group
// j & 1 has read tile j, so the two groups run half a tile apart and each
// DMA burst is one image.  Every wait polls with s_sleep and gives up after
// 2^16 polls, ~2 ms (wrong results, never a hung GPU).
__device__ __forceinline__ uint32_t lds_poll(const uint32_t P2P_LDS* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_wait_ge(const uint32_t P2P_LDS* p, uint32_t target) {
  for (int spin = 0; lds_poll(p) < target && spin < (1 << 16); ++spin) __builtin_amdgcn_s_sleep(1);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void lds_signal(uint32_t P2P_LDS* p) {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int RULE, int MODE, bool SEGS>
__global__ __launch_bounds__(768) void robust_lds_g2a_kernel(const float* const* __restrict__ peers,
                                                             const Seg* __restrict__ segs, int nseg,
                                                             int64_t ntiles, int K, int trim_b, int64_t n,
                                                             float* w, float* out, float lr) {
  constexpr int L = 4, H = 64;
  using Lay = LdsLayout<L, H>;
  static_assert(Lay::NBUF == 2 && Lay::W == 4 && Lay::BYTES + 16 <= 160 * 1024, "one image per sorter group");
  __shared__ __attribute__((aligned(16))) uint8_t lds_raw[Lay::BYTES + 16];
  uint8_t P2P_LDS* lds = (uint8_t P2P_LDS*)lds_raw;
  uint32_t P2P_LDS* full = (uint32_t P2P_LDS*)(lds + Lay::BYTES);  // full[0..1], empty[0..1]
  uint32_t P2P_LDS* empty = full + 2;
  const int wi = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  const bool loader = wi >= 2 * Lay::W;
  const int g = loader ? 0 : wi / Lay::W;
  const int li = wi - 2 * Lay::W;
  const int q = lane % L, c = (wi % Lay::W) * Lay::TW + lane / L;

  const int64_t nb = gridDim.x;
  int64_t t0 = blockIdx.x;
  if ((nb & 7) == 0) t0 = (blockIdx.x & 7) * (nb >> 3) + (blockIdx.x >> 3);
  if (t0 >= ntiles) return;  // block-uniform
  const int64_t m = ceil_div(ntiles - t0, nb);  // this block's tiles: t0 + j*nb, j < m
  if (threadIdx.x < 4) full[threadIdx.x] = 0;
  __syncthreads();

  const float* rp[Lay::NCHW];
  int64_t cur_seg = -1;
  bool aligned = false;
  auto row_of = [&](int mm) {
    const int ch = li * Lay::NCHW + mm;
    const int row = (ch / Lay::CPS) * H + (ch % Lay::CPS) * Lay::RPP + lane / Lay::LPR;
    return row < K ? row : K - 1;
  };
  auto bind = [&](const TileSrc& s) {
    if (s.seg == cur_seg) return;
    cur_seg = s.seg;
    aligned = all_aligned16(s.peers, K, s.w, nullptr);
    if (loader) {
#pragma unroll
      for (int mm = 0; mm < Lay::NCHW; ++mm) rp[mm] = table_at(s.peers, row_of(mm));
    }
  };
  auto src_of = [&](int64_t j, bool& dma) {
    const TileSrc s = locate<Lay::TB, SEGS>(peers, segs, nseg, n, w, out, t0 + j * nb);
    bind(s);
    dma = aligned && s.c0 + Lay::TB <= s.n;
    return s;
  };
  auto real_piece = [&](int mm) {
    const int ch = li * Lay::NCHW + mm;
    return MODE != 0 || (ch / Lay::CPS) * H + (ch % Lay::CPS) * Lay::RPP < K;
  };
  auto npieces = [&](const TileSrc& s) {
    int np = 0;
#pragma unroll
    for (int mm = 0; mm < Lay::NCHW; ++mm) np += real_piece(mm) ? 1 : 0;
    return np + ((s.w && li == 0) ? 1 : 0);
  };
  auto issue = [&](const TileSrc& s, int img_off) {
    uint8_t P2P_LDS* im = lds + img_off;
    const int64_t off = s.c0 + 4 * (lane % Lay::LPR);
#pragma unroll
    for (int mm = 0; mm < Lay::NCHW; ++mm) {
      const int ch = li * Lay::NCHW + mm;
      if (real_piece(mm)) glds16(rp[mm] + off, im + (ch / Lay::CPS) * Lay::SB + (ch % Lay::CPS) * 1024);
    }
    if (s.w && li == 0 && lane < Lay::LPR) glds16(s.w + s.c0 + 4 * lane, im + Lay::WOFF);
  };

  if (loader) {
    // pieces in flight per tile j (0 when tile j is not DMA'd)
    int np_cur = 0, np_nxt = 0;
    bool dma;
    {
      const TileSrc s = src_of(0, dma);
      if (dma) { issue(s, 0); np_cur = npieces(s); }
    }
    if (m > 1) {
      const TileSrc s = src_of(1, dma);
      if (dma) { issue(s, Lay::IMG); np_nxt = npieces(s); }
    }
    for (int64_t j = 0; j < m; ++j) {
      wait_vmcnt(np_nxt);  // this loader's pieces of tile j have landed (tile j+1's may not)
      if (np_cur) {
        asm volatile("" ::: "memory");
        if (lane == 0) __hip_atomic_fetch_add(&full[j & 1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      int np_new = 0;
      if (j + 2 < m) {
        lds_wait_ge(&empty[j & 1], static_cast<uint32_t>(4 * (j / 2 + 1)));  // group j&1 has read tile j
        const TileSrc s = src_of(j + 2, dma);
        if (dma) { issue(s, (j & 1) * Lay::IMG); np_new = npieces(s); }
      }
      np_cur = np_nxt;
      np_nxt = np_new;
    }
    return;
  }
  uint8_t P2P_LDS* im = lds + g * Lay::IMG;
  uint32_t dma_seen = 0;  // DMA'd tiles of this group so far
  for (int64_t j = g; j < m; j += 2) {
    bool dma;
    const TileSrc me = src_of(j, dma);
    if (dma) {
      ++dma_seen;
      lds_wait_ge(&full[g], 4 * dma_seen);  // all four loaders' pieces landed
    } else {
      fill_direct<L, H>(im, me.peers, me.w, me.n, me.c0 + c, K, q, c);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    uint32_t v[H];
    const uint32_t P2P_LDS* sl = (const uint32_t P2P_LDS*)(im + q * Lay::SB) + c;
#pragma unroll
    for (int jj = 0; jj < H; ++jj) v[jj] = sl[jj * (Lay::RB / 4)];
    const float wv = me.w ? ((const float P2P_LDS*)(im + Lay::WOFF))[c] : 0.f;
    lds_signal(&empty[g]);  // this wave's reads are done: image free once all 4 signal
    bool own = false;
    float agg;
    bool fast = false;  // NaN-free wave with every slot real: the float network
    if constexpr (MODE != 0) fast = !wave_has_nan(v);
    if (fast) {
      fk f[H];
#pragma unroll
      for (int jj = 0; jj < H; ++jj) f[jj].x = __uint_as_float(v[jj]);
      agg = reduce_keys<L, H, RULE, MODE>(f, q, K, trim_b, own);
    } else {
#pragma unroll
      for (int jj = 0; jj < H; ++jj) {
        const bool real = (MODE != 0) || (q * H + jj < K);
        v[jj] = real ? f2key(v[jj]) : 0xFFFFFFFFu;
      }
      agg = reduce_keys<L, H, RULE, MODE>(v, q, K, trim_b, own);
    }
    const int64_t e = me.c0 + c;
    if (own && e < me.n) {
      if (me.out) stg(me.out + e, agg);
      if (me.w) stg(me.w + e, apply_lr(wv, lr, agg));
    }
  }
}

template <int RULE, int MODE, bool SEGS>
static void launch_lds_g2a_kernel(const LdsArgs& a) {
  using Lay = LdsLayout<4, 64>;
  auto kern = robust_lds_g2a_kernel<RULE, MODE, SEGS>;
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
                     ntiles, a.K, a.trim_b, a.n, a.w, a.out, a.lr);
}

template <int RULE>
static void launch_lds_g2a(const LdsArgs& a) {
  constexpr int KP = 256;
  const bool special = RULE == P2P_RULE_MEDIAN ? a.K == KP : (a.K == KP && a.trim_b == (KP * 2) / 10);
  if (special) {
    if (a.segs) launch_lds_g2a_kernel<RULE, RULE == P2P_RULE_MEDIAN ? 1 : 2, true>(a);
    else launch_lds_g2a_kernel<RULE, RULE == P2P_RULE_MEDIAN ? 1 : 2, false>(a);
  } else {
    if (a.segs) launch_lds_g2a_kernel<RULE, 0, true>(a);
    else launch_lds_g2a_kernel<RULE, 0, false>(a);
  }
}

}  // namespace p2p

// variant: 0 the 4-lane layout (4 lanes x 64 keys), 2 LDS 4 x 32 (K <= 128), 3 LDS 2 x 64 (K <= 128),
// 4 LDS 1 x 128 (K <= 128), 5 LDS 2 x 128 (K in 129..256), 7 two sorter groups per
// block (K in 129..256), 8 the same, asynchronous (LDS counters); the
// self-staged layout (variant 6, profiles/r02/ab/labself*) and the radix16
// affine median (variant 1) were removed
extern "C" int32_t p2p_lab_robust(int32_t variant, const float* const* peers, int32_t k, int64_t n,
                                  int32_t rule, int32_t trim_b, float lr, float* w, float* out,
                                  p2p_stream_t stream) {
  LdsArgs a{peers, nullptr, 0, 0, k, trim_b, n, w, out, lr, static_cast<hipStream_t>(stream)};
  const bool med = rule == P2P_RULE_MEDIAN;
  switch (variant) {
    case 0:
      if (med) launch_lds<4, 64, P2P_RULE_MEDIAN>(a); else launch_lds<4, 64, P2P_RULE_TRIMMED>(a);
      break;
    case 2:
      if (k > 128) return P2P_ERR_UNSUPPORTED;
      if (med) launch_lds<4, 32, P2P_RULE_MEDIAN>(a); else launch_lds<4, 32, P2P_RULE_TRIMMED>(a);
      break;
    case 3:
      if (k > 128) return P2P_ERR_UNSUPPORTED;
      if (med) launch_lds<2, 64, P2P_RULE_MEDIAN>(a); else launch_lds<2, 64, P2P_RULE_TRIMMED>(a);
      break;
    case 4:
      if (k > 128) return P2P_ERR_UNSUPPORTED;
      if (med) launch_lds<1, 128, P2P_RULE_MEDIAN>(a); else launch_lds<1, 128, P2P_RULE_TRIMMED>(a);
      break;
    case 5:  // 2 lanes x 128 keys per coordinate (one LDS image of 128 coordinates)
      if (k <= 128) return P2P_ERR_UNSUPPORTED;
      if (med) launch_lds<2, 128, P2P_RULE_MEDIAN>(a); else launch_lds<2, 128, P2P_RULE_TRIMMED>(a);
      break;
    case 7:  // two sorter groups per block (12 waves: 2 x 4 sorters + 4 loaders), key network
      if (k <= 128) return P2P_ERR_UNSUPPORTED;
      if (med) launch_lds_g2<P2P_RULE_MEDIAN>(a); else launch_lds_g2<P2P_RULE_TRIMMED>(a);
      break;
    case 8:  // two sorter groups per block, asynchronous (LDS counters instead of barriers)
      if (k <= 128) return P2P_ERR_UNSUPPORTED;
      if (med) launch_lds_g2a<P2P_RULE_MEDIAN>(a); else launch_lds_g2a<P2P_RULE_TRIMMED>(a);
      break;
    default:
      return P2P_ERR_INVALID;
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? P2P_OK : static_cast<int32_t>(e);
}
