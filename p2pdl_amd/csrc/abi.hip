// C-ABI front door: version, error text, rule dispatch (include/p2pdl.h).
#include "p2p_common.h"

extern "C" int64_t p2p_fedavg_tile_elems(void);
extern "C" int64_t p2p_robust_tile_elems(int32_t rule, int32_t k);
extern "C" int32_t p2p_fedavg_segments_f32(const p2p_segment_t* segs, int32_t nseg,
                                           int64_t total_tiles, int32_t k, float lr,
                                           p2p_stream_t stream, int32_t recip);
extern "C" int32_t p2p_robust_dispatch(const float* const* peers, const p2p_segment_t* segs,
                                       int32_t nseg, int64_t tiles, int32_t k, int32_t rule,
                                       int32_t trim_b, int64_t n, float* w, float* out, float lr,
                                       p2p_stream_t stream);

int32_t p2p_fedavg_flat_launch(const float* const* peers, int32_t k, int64_t n, float* w, float* out,
                               float lr, p2p_stream_t stream, int32_t recip, int32_t hints);

static bool is_fedavg(int32_t rule) { return rule == P2P_RULE_FEDAVG || rule == P2P_RULE_FEDAVG_TORCH_GPU; }

extern "C" int32_t p2p_abi_version(void) { return P2P_ABI_VERSION; }

extern "C" const char* p2p_strerror(int32_t code) {
  switch (code) {
    case P2P_OK: return "ok";
    case P2P_ERR_INVALID: return "p2p: invalid argument";
    case P2P_ERR_UNSUPPORTED: return "p2p: unsupported (robust rules need 1 <= k <= 256)";
    case P2P_ERR_ALIGN: return "p2p: float pointer not 4-byte aligned";
    default: break;
  }
  if (code > 0) return hipGetErrorString(static_cast<hipError_t>(code));
  return "p2p: unknown error";
}

extern "C" int64_t p2p_tile_elems(int32_t rule, int32_t k) {
  return is_fedavg(rule) ? p2p_fedavg_tile_elems() : p2p_robust_tile_elems(rule, k);
}

static bool misaligned4(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 3) != 0; }

extern "C" int32_t p2p_median_f32(const float* const* peers, int32_t k, int64_t n, float* out,
                                  p2p_stream_t stream) {
  if (!peers || !out || n < 0) return P2P_ERR_INVALID;
  if (misaligned4(out)) return P2P_ERR_ALIGN;
  if (n == 0) return k < 1 ? P2P_ERR_INVALID : P2P_OK;
  return p2p_robust_dispatch(peers, nullptr, 0, 0, k, P2P_RULE_MEDIAN, 0, n, nullptr, out, 0.f, stream);
}

extern "C" int32_t p2p_trimmed_mean_f32(const float* const* peers, int32_t k, int64_t n,
                                        int32_t trim_b, float* out, p2p_stream_t stream) {
  if (!peers || !out || n < 0) return P2P_ERR_INVALID;
  if (misaligned4(out)) return P2P_ERR_ALIGN;
  if (n == 0) return (k < 1 || trim_b < 0 || k - 2 * trim_b <= 0) ? P2P_ERR_INVALID : P2P_OK;
  return p2p_robust_dispatch(peers, nullptr, 0, 0, k, P2P_RULE_TRIMMED, trim_b, n, nullptr, out, 0.f,
                             stream);
}

extern "C" int32_t p2p_aggregate_ex_f32(const float* const* peers, int32_t k, int64_t n, int32_t rule,
                                        int32_t trim_b, float lr, float* w, float* out, int32_t hints,
                                        p2p_stream_t stream) {
  if (!peers || (!w && !out) || k < 1 || n < 0 || (hints & ~P2P_HINT_SHARE_CUS)) return P2P_ERR_INVALID;
  if (misaligned4(w) || misaligned4(out)) return P2P_ERR_ALIGN;
  if (is_fedavg(rule)) {
    if (n == 0) return P2P_OK;
    return p2p_fedavg_flat_launch(peers, k, n, w, out, lr, stream, rule == P2P_RULE_FEDAVG_TORCH_GPU, hints);
  }
  if (rule != P2P_RULE_MEDIAN && rule != P2P_RULE_TRIMMED) return P2P_ERR_INVALID;
  if (rule == P2P_RULE_TRIMMED && (trim_b < 0 || k - 2 * trim_b <= 0)) return P2P_ERR_INVALID;
  if (n == 0) return k > 256 ? P2P_ERR_UNSUPPORTED : P2P_OK;
  return p2p_robust_dispatch(peers, nullptr, 0, 0, k, rule, trim_b, n, w, out, lr, stream);
}

extern "C" int32_t p2p_aggregate_f32(const float* const* peers, int32_t k, int64_t n, int32_t rule,
                                     int32_t trim_b, float lr, float* w, float* out,
                                     p2p_stream_t stream) {
  return p2p_aggregate_ex_f32(peers, k, n, rule, trim_b, lr, w, out, 0, stream);
}

extern "C" int32_t p2p_aggregate_segments_f32(const p2p_segment_t* segs, int32_t nseg,
                                              int64_t total_tiles, int32_t k, int32_t rule,
                                              int32_t trim_b, float lr, p2p_stream_t stream) {
  if (!segs || nseg < 1 || k < 1 || total_tiles < 0) return P2P_ERR_INVALID;
  if (total_tiles > 0x7FFFFFFFll) return P2P_ERR_UNSUPPORTED;
  if (is_fedavg(rule))
    return p2p_fedavg_segments_f32(segs, nseg, total_tiles, k, lr, stream, rule == P2P_RULE_FEDAVG_TORCH_GPU);
  if (rule != P2P_RULE_MEDIAN && rule != P2P_RULE_TRIMMED) return P2P_ERR_INVALID;
  if (total_tiles == 0) return P2P_OK;
  return p2p_robust_dispatch(nullptr, segs, nseg, total_tiles, k, rule, trim_b, 0, nullptr, nullptr, lr,
                             stream);
}
