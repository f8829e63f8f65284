// K1 for float16 / bfloat16 models (reference aggregator/aggregation.py:15-38
// on a model whose state_dict is half precision, e.g. after model.half()).
//
// torch runs every op of the reference's loop in float32 and rounds the
// result to the storage type, so the exact restatement is, per coordinate:
//   acc = +0                                  (:15)
//   acc = r(acc + u_k), k in list order       (:25-28)
//   acc = r(acc / K)   [GPU rule: r(acc * fl(1/K))]   (:31-32)
//   w   = r(w + r(fp32(lr) * acc))            (:36-38)
// with r() round-to-nearest-even to float16 / bfloat16 (torch's conversions;
// a NaN stays a NaN).  2(K+2) bytes per coordinate, HBM-bound like
// the fp32 kernel; each lane handles 8 consecutive coordinates per step with
// one 16-byte load per peer (one 1-KiB wave instruction), 4 peers in flight.
#include "p2p_common.h"

namespace p2p {

template <int DT>
__device__ __forceinline__ float f16_to_f32(uint16_t b) {
  if constexpr (DT == P2P_DTYPE_F16) {
    _Float16 h;
    __builtin_memcpy(&h, &b, 2);
    return static_cast<float>(h);
  } else {
    return __uint_as_float(static_cast<uint32_t>(b) << 16);
  }
}

template <int DT>
__device__ __forceinline__ uint16_t f32_to_16(float x) {
  if constexpr (DT == P2P_DTYPE_F16) {
    const _Float16 h = static_cast<_Float16>(x);  // v_cvt_f16_f32: round to nearest even
    uint16_t b;
    __builtin_memcpy(&b, &h, 2);
    return b;
  } else {  // c10::BFloat16's round_to_nearest_even
    const uint32_t u = __float_as_uint(x);
    if (x != x) return 0x7FC0;
    return static_cast<uint16_t>((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
  }
}

// The fp32 result first, then the storage rounding -- as torch does.  The
// empty asm pins the fp32 value: without it the backend folds
// fptrunc(fmul(lr, m)) into one v_fma_mixlo_f16, a single rounding of the
// exact product to f16, which differs from fp32-then-f16 (measured: 3 of
// 200k MLP coordinates, one f16 ulp).
__device__ __forceinline__ float pin(float x) {
  asm volatile("" : "+v"(x));
  return x;
}

template <int DT>
__device__ __forceinline__ float rnd(float x) { return f16_to_f32<DT>(f32_to_16<DT>(pin(x))); }

// RECIP (P2P_RULE_FEDAVG_TORCH_GPU): acc * fl(1/K), as torch's GPU kernels
// divide by a CPU scalar.  Every op fp32-then-storage, as torch's vectorized
// GPU path computes (its non-vectorized path single-rounds float16 products
// through v_fma_mixlo_f16 -- a few midpoint coordinates of small tensors,
// tools/torch_half_probe.py, tests/test_fedavg16.py -- a property of torch's
// code path, not of the values).
template <int DT, bool RECIP>
__device__ __forceinline__ uint16_t fedavg16_one(float acc, float fk, float inv, float lr, uint16_t w) {
  const float m = rnd<DT>(RECIP ? __fmul_rn(acc, inv) : acc / fk);
  const float t = rnd<DT>(__fmul_rn(lr, m));
  return f32_to_16<DT>(pin(__fadd_rn(f16_to_f32<DT>(w), t)));
}

typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
constexpr int kV16 = 8;       // coordinates per lane per step: one 16-byte load per peer (1 KiB per wave)
constexpr int kU16 = 4;       // peer loads in flight per lane before the rounding chain consumes them

template <int DT, bool RECIP>
__global__ __launch_bounds__(kBlock) void fedavg16_kernel(const uint16_t* const* __restrict__ peers, int K,
                                                          int64_t n, uint16_t* w, float lr) {
  uintptr_t a = reinterpret_cast<uintptr_t>(w);  // 16-byte vector loads need every buffer 16-byte aligned
  for (int k = 0; k < K; ++k) a |= reinterpret_cast<uintptr_t>(table_at(peers, k));
  const bool vec = (a & 15) == 0;
  const float fk = static_cast<float>(K);
  const float inv = RECIP ? 1.0f / fk : 0.f;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock * kV16;
  for (int64_t i = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) * kV16; i < n; i += stride) {
    if (vec && i + kV16 <= n) {
      float acc[kV16];
#pragma unroll
      for (int e = 0; e < kV16; ++e) acc[e] = 0.f;
      int k = 0;
      for (; k + kU16 <= K; k += kU16) {
        u16x8 u[kU16];
#pragma unroll
        for (int j = 0; j < kU16; ++j) u[j] = ldg_nt(reinterpret_cast<const u16x8*>(table_at(peers, k + j) + i));
#pragma unroll
        for (int j = 0; j < kU16; ++j)  // strictly in list order (:25-28)
#pragma unroll
          for (int e = 0; e < kV16; ++e) acc[e] = rnd<DT>(__fadd_rn(acc[e], f16_to_f32<DT>(u[j][e])));
      }
      for (; k < K; ++k) {
        const u16x8 u = ldg_nt(reinterpret_cast<const u16x8*>(table_at(peers, k) + i));
#pragma unroll
        for (int e = 0; e < kV16; ++e) acc[e] = rnd<DT>(__fadd_rn(acc[e], f16_to_f32<DT>(u[e])));
      }
      const u16x8 wv = ldg(reinterpret_cast<const u16x8*>(w + i));
      u16x8 o;
#pragma unroll
      for (int e = 0; e < kV16; ++e) o[e] = fedavg16_one<DT, RECIP>(acc[e], fk, inv, lr, wv[e]);
      stg(reinterpret_cast<u16x8*>(w + i), o);
    } else {
      for (int64_t j = i; j < n && j < i + kV16; ++j) {
        float acc = 0.f;
        for (int k = 0; k < K; ++k) acc = rnd<DT>(__fadd_rn(acc, f16_to_f32<DT>(ldg(table_at(peers, k) + j))));
        stg(w + j, fedavg16_one<DT, RECIP>(acc, fk, inv, lr, ldg(w + j)));
      }
    }
  }
}

}  // namespace p2p

using namespace p2p;

extern "C" int32_t p2p_fedavg_apply_16(const uint16_t* const* peers, int32_t k, int64_t n, uint16_t* w, float lr,
                                       int32_t dtype, int32_t rule, p2p_stream_t stream) {
  if (!peers || !w || k < 1 || n < 0) return P2P_ERR_INVALID;
  if (dtype != P2P_DTYPE_F16 && dtype != P2P_DTYPE_BF16) return P2P_ERR_INVALID;
  if (rule != P2P_RULE_FEDAVG && rule != P2P_RULE_FEDAVG_TORCH_GPU) return P2P_ERR_INVALID;
  if (reinterpret_cast<uintptr_t>(w) & 1) return P2P_ERR_ALIGN;
  if (n == 0) return P2P_OK;
  const int64_t groups = ceil_div(n, kV16);
  const int64_t blocks = ceil_div(groups, kBlock);
  const unsigned grid = static_cast<unsigned>(blocks < 256 * 8 ? blocks : 256 * 8);
  const hipStream_t s = static_cast<hipStream_t>(stream);
  const bool recip = rule == P2P_RULE_FEDAVG_TORCH_GPU;
  if (dtype == P2P_DTYPE_F16) {
    if (recip) hipLaunchKernelGGL((fedavg16_kernel<P2P_DTYPE_F16, true>), dim3(grid), dim3(kBlock), 0, s, peers, k, n, w, lr);
    else hipLaunchKernelGGL((fedavg16_kernel<P2P_DTYPE_F16, false>), dim3(grid), dim3(kBlock), 0, s, peers, k, n, w, lr);
  } else {
    if (recip) hipLaunchKernelGGL((fedavg16_kernel<P2P_DTYPE_BF16, true>), dim3(grid), dim3(kBlock), 0, s, peers, k, n, w, lr);
    else hipLaunchKernelGGL((fedavg16_kernel<P2P_DTYPE_BF16, false>), dim3(grid), dim3(kBlock), 0, s, peers, k, n, w, lr);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? P2P_OK : static_cast<int32_t>(e);
}
