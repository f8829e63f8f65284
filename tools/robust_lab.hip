// A/B library for the robust kernels -- NOT the product.  It compiles the
// product's robust_lds.hip with P2P_LAB (fallback counters) and exposes the
// template instantiations the product dispatch does not use, so variants can
// be timed and bit-compared against the product kernel on the same inputs.
// Built by `make -C p2pdl_amd/csrc lab` into tools/libp2pdl_lab.so (the
// product objects minus robust_lds.o, plus this file); selected with
// P2P_LIB=tools/libp2pdl_lab.so by tools/lab_robust.py.
#include "../p2pdl_amd/csrc/robust_lds.hip"

using namespace p2p;

// variant: 0 product layout (4 lanes x 64 keys), 1 radix16 affine median
// (K = 256 only), 2 LDS 4 x 32 (K <= 128), 3 LDS 2 x 64 (K <= 128),
// 4 LDS 1 x 128 (K <= 128), 5 LDS 2 x 128 (K in 129..256), 6 self-staged 4 x 64
// (no loader waves, one image, two blocks per CU; K in 129..256), 7 two sorter
// groups per block (K in 129..256)
extern "C" int32_t p2p_lab_robust(int32_t variant, const float* const* peers, int32_t k, int64_t n,
                                  int32_t rule, int32_t trim_b, float lr, float* w, float* out,
                                  p2p_stream_t stream) {
  LdsArgs a{peers, nullptr, 0, 0, k, trim_b, n, w, out, lr, static_cast<hipStream_t>(stream)};
  const bool med = rule == P2P_RULE_MEDIAN;
  switch (variant) {
    case 0:
      if (med) launch_lds<4, 64, P2P_RULE_MEDIAN>(a); else launch_lds<4, 64, P2P_RULE_TRIMMED>(a);
      break;
    case 1:
      if (!med || k != 256) return P2P_ERR_UNSUPPORTED;
      launch_lds_kernel<4, 64, P2P_RULE_MEDIAN, 1, false, 0, 2>(a);
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
    case 6:  // self-staged: 4 waves sort AND issue the DMA, one image, two blocks per CU
      if (k <= 128) return P2P_ERR_UNSUPPORTED;
      if (med) launch_lds<4, 64, P2P_RULE_MEDIAN, 1, true>(a); else launch_lds<4, 64, P2P_RULE_TRIMMED, 1, true>(a);
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

// Waves that took the exact fallback since the last reset (radix16 variant).
extern "C" int64_t p2p_lab_fallbacks(int32_t reset) {
  int h[64];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_lab_fallback), sizeof(h)) != hipSuccess) return -1;
  if (reset) {
    int z[64] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_lab_fallback), z, sizeof(z)) != hipSuccess) return -1;
  }
  return h[0];
}
