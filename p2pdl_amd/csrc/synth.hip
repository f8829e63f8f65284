// Synthetic inputs on device: a counter PRNG that the CPU
// oracle restates bit for bit, so benchmark inputs are reproducible on host
// and are generated in HBM outside any timed region (no host->device copy).
#include "p2p_common.h"

namespace p2p {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ __launch_bounds__(kBlock) void synth_kernel(float* out, int64_t n, uint64_t seed,
                                                       uint32_t peer, float scale, int64_t chunk,
                                                       int nranks, int rank) {
  const uint64_t key = seed ^ (static_cast<uint64_t>(peer) << 40);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
    int64_t g = i;
    if (nranks > 1 && chunk > 0) {
      const int64_t s = i / chunk;
      g = (s * nranks + rank) * chunk + (i - s * chunk);
    }
    const uint64_t u = splitmix64(key ^ static_cast<uint64_t>(g)) >> 40;
    const float x = __fsub_rn(__fmul_rn(static_cast<float>(u), 0x1p-23f), 1.0f);
    out[i] = __fmul_rn(x, scale);
  }
}

}  // namespace p2p

using namespace p2p;

extern "C" int32_t p2p_fill_synthetic_f32(float* out, int64_t n, uint64_t seed, int32_t peer,
                                          float scale, int64_t chunk, int32_t nranks, int32_t rank,
                                          p2p_stream_t stream) {
  if (!out || n < 0) return P2P_ERR_INVALID;
  if (n == 0) return P2P_OK;
  const int64_t blocks = ceil_div(n, kBlock);
  const unsigned grid = static_cast<unsigned>(blocks < 256 * 16 ? blocks : 256 * 16);
  hipLaunchKernelGGL(synth_kernel, dim3(grid), dim3(kBlock), 0, static_cast<hipStream_t>(stream), out,
                     n, seed, static_cast<uint32_t>(peer), scale, chunk, nranks, rank);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? P2P_OK : static_cast<int32_t>(e);
}
