// K3 -- batched SHA-256 (FIPS 180-4) over serialized peer updates, gfx950.
//
// The reference hashes every serialized update inside ECDSA(SHA256()):
// sign_data at utils/crypto.py:54-57 and verify_signature at :92-96, over the
// bytes of pickle.dumps(local_update) (node/node.py:285).  Each message is a
// serial Merkle-Damgard chain, so the only parallelism is across messages:
// one lane owns one message and runs its compression chain in VGPRs.  The
// round function uses gfx950's 3-input ops (v_bitop3_b32 for the Sigma XORs
// and Ch / Maj, v_add3_u32 for the sums, v_alignbit_b32 rotates).  With 256
// messages only 4 waves carry chains, and a lone wave issues about one
// instruction per ~5.5 cycles (profiles/r01/probes), so a block costs
// (instructions on the chain) x 5.5 cycles: the schedule expansion is moved
// to a second wave (sha256_pair_kernel).  Bounded by per-wave serial issue,
// not by HBM; DESIGN.md prices it.
#include "p2p_common.h"

namespace p2p {

__constant__ uint32_t kK256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t rotr(uint32_t x, int r) { return __builtin_rotateright32(x, r); }
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }
// a ^ b ^ c in one v_bitop3_b32 (truth table 0x96); hipcc emits two v_xor_b32
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Byte j (0..63) of the padded tail region of a message of `len` bytes whose
// full 64-B blocks are already consumed; `tail` points at the first tail byte.
__device__ __forceinline__ uint32_t tail_byte(const uint8_t* tail, uint32_t rem, uint32_t j,
                                              uint32_t nblk, uint64_t bits) {
  if (j < rem) return ldg(tail + j);
  if (j == rem) return 0x80u;
  const uint32_t end = 64u * nblk;
  if (j >= end - 8u) return static_cast<uint32_t>(bits >> (8u * (end - 1u - j))) & 0xFFu;
  return 0u;
}

// Message schedule of one block, K folded in: kw[t] = K[t] + W[t].
__device__ __forceinline__ void schedule_kw(uint32_t (&W)[64]) {
#pragma unroll
  for (int t = 16; t < 64; ++t) {
    const uint32_t w15 = W[t - 15], w2 = W[t - 2];
    const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
    const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
    W[t] = W[t - 16] + s0 + W[t - 7] + s1;
  }
#pragma unroll
  for (int t = 0; t < 64; ++t) W[t] += kK256[t];
}

// 64 rounds with the schedule already expanded (kw = K + W).
__device__ __forceinline__ void rounds_kw(uint32_t (&h)[8], const uint32_t (&kw)[64]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int t = 0; t < 64; ++t) {
    const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
    const uint32_t ch = __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);  // e ? f : g
    const uint32_t T1 = hh + S1 + ch + kw[t];
    const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
    const uint32_t mj = __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);  // majority
    hh = g; g = f; f = e; e = d + T1; d = c; c = b; b = a; a = T1 + S0 + mj;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// Words 0..15 of block `blk` of a message (message blocks, then the 1 or 2
// padding blocks: 0x80, zeros, 64-bit big-endian bit length).
__device__ __forceinline__ void load_block(uint32_t (&W)[64], const uint8_t* m, uint64_t len, uint64_t blk,
                                           bool al16) {
  const uint64_t full = len >> 6;
  if (blk < full) {
    const uint8_t* p = m + (blk << 6);
    if (al16) {
      const u32x4* q = reinterpret_cast<const u32x4*>(p);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const u32x4 x = ldg_nt(q + j);
        W[4 * j] = bswap(x.x); W[4 * j + 1] = bswap(x.y);
        W[4 * j + 2] = bswap(x.z); W[4 * j + 3] = bswap(x.w);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j)
        W[j] = (uint32_t(ldg(p + 4 * j)) << 24) | (uint32_t(ldg(p + 4 * j + 1)) << 16) |
               (uint32_t(ldg(p + 4 * j + 2)) << 8) | uint32_t(ldg(p + 4 * j + 3));
    }
    return;
  }
  const uint32_t rem = static_cast<uint32_t>(len & 63);
  const uint32_t nblk = (rem + 9u <= 64u) ? 1u : 2u;
  const uint8_t* tail = m + (full << 6);
  const uint64_t bits = len * 8u;
  const uint32_t tb = static_cast<uint32_t>(blk - full);
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t o = tb * 64u + 4u * j;
    W[j] = (tail_byte(tail, rem, o, nblk, bits) << 24) | (tail_byte(tail, rem, o + 1, nblk, bits) << 16) |
           (tail_byte(tail, rem, o + 2, nblk, bits) << 8) | tail_byte(tail, rem, o + 3, nblk, bits);
  }
}

__device__ __forceinline__ uint64_t blocks_of(uint64_t len) {
  return (len >> 6) + (((len & 63) + 9u <= 64u) ? 1u : 2u);
}

// Workgroup = 2 waves over the same 64 messages (lane = message).  A lone
// wave issues about one instruction per ~5.5 cycles, so each message's chain
// is issue-bound: the 64 rounds stay on wave 0 (14 instructions per round
// with K+W precomputed), while wave 1 loads, byte-swaps and expands the
// schedule of the NEXT block (~560 instructions) and hands K+W over through
// a double-buffered LDS ring ([t/4][lane][4] u32: ds_*_b128, conflict-free).
// One barrier per block.  Lanes whose message has fewer blocks idle (exec).
constexpr int kShaLanes = 64;
__global__ __launch_bounds__(128) void sha256_pair_kernel(const uint8_t* const* __restrict__ msgs,
                                                          const uint64_t* __restrict__ lens, int k,
                                                          uint8_t* __restrict__ digests) {
  __shared__ __attribute__((aligned(16))) u32x4 ring[3][16][kShaLanes];
  const int wi = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * kShaLanes + lane;
  const bool live = i < k;
  const uint8_t* m = live ? ldg(msgs + i) : nullptr;
  const uint64_t len = live ? ldg(lens + i) : 0;
  const uint64_t nb = live ? blocks_of(len) : 0;
  // wave-uniform block count: max over the 64 lanes (same in both waves)
  uint64_t nmax = nb;
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) {
    const uint32_t lo = __shfl_xor(static_cast<uint32_t>(nmax), s, 64);
    const uint32_t hi = __shfl_xor(static_cast<uint32_t>(nmax >> 32), s, 64);
    const uint64_t o = (static_cast<uint64_t>(hi) << 32) | lo;
    nmax = o > nmax ? o : nmax;
  }
  nmax = uniform_u64(nmax);
  const bool al16 = (reinterpret_cast<uintptr_t>(m) & 15) == 0;

  // Three-slot ring, ONE barrier per block: before barrier j the schedule
  // wave has expanded block j+2 (and written blocks <= j+1); after it, it
  // stores block j+2 while the round wave issues the LDS reads of block j+1
  // and then runs block j's rounds from registers -- the read latency hides
  // behind 64 rounds and block j's K+W never waits on the ring.
  auto put = [&](int slot, const uint32_t (&W)[64]) {
#pragma unroll
    for (int q = 0; q < 16; ++q) ring[slot][q][lane] = u32x4{W[4 * q], W[4 * q + 1], W[4 * q + 2], W[4 * q + 3]};
  };
  auto get = [&](int slot, uint32_t (&kw)[64]) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const u32x4 x = ring[slot][q][lane];
      kw[4 * q] = x.x; kw[4 * q + 1] = x.y; kw[4 * q + 2] = x.z; kw[4 * q + 3] = x.w;
    }
  };
  if (wi == 1) {  // schedule wave
    for (uint64_t j = 0; j < 2 && j < nb; ++j) {
      uint32_t W[64];
      load_block(W, m, len, j, al16);
      schedule_kw(W);
      put(static_cast<int>(j), W);
    }
    __syncthreads();  // blocks 0 and 1 are in the ring
    for (uint64_t j = 0; j < nmax; ++j) {
      uint32_t W[64];
      const bool more = j + 2 < nb;
      if (more) {
        load_block(W, m, len, j + 2, al16);
        schedule_kw(W);
      }
      __syncthreads();  // barrier j: slot (j+2)%3 (block j-1) has been read
      if (more) put(static_cast<int>((j + 2) % 3), W);
    }
    return;
  }
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint32_t kwa[64], kwb[64];
  __syncthreads();  // blocks 0 and 1 are in the ring
  if (nb > 0) get(0, kwa);
  for (uint64_t j = 0; j < nmax; j += 2) {  // two blocks per trip: kwa / kwb alternate
    __syncthreads();  // barrier j: block j+1 is in slot (j+1)%3
    if (j + 1 < nb) get(static_cast<int>((j + 1) % 3), kwb);
    if (j < nb) rounds_kw(h, kwa);
    if (j + 1 >= nmax) break;
    __syncthreads();  // barrier j+1
    if (j + 2 < nb) get(static_cast<int>((j + 2) % 3), kwa);
    if (j + 1 < nb) rounds_kw(h, kwb);
  }
  if (live) {
    uint4* d = reinterpret_cast<uint4*>(digests + 32 * static_cast<int64_t>(i));
    d[0] = make_uint4(bswap(h[0]), bswap(h[1]), bswap(h[2]), bswap(h[3]));
    d[1] = make_uint4(bswap(h[4]), bswap(h[5]), bswap(h[6]), bswap(h[7]));
  }
}

// Order-preserving compaction of accepted payload pointers (single block).
__global__ __launch_bounds__(256) void accept_kernel(const uint8_t* __restrict__ digests,
                                                     const uint8_t* __restrict__ expected,
                                                     const float* const* __restrict__ payloads, int k,
                                                     const float** accepted, int32_t* count) {
  __shared__ int32_t scan[256];
  int32_t carry = 0;
  for (int base = 0; base < k; base += 256) {
    const int i = base + threadIdx.x;
    int32_t ok = 0;
    if (i < k) {
      const uint4* a = reinterpret_cast<const uint4*>(digests + 32 * static_cast<int64_t>(i));
      const uint4* b = reinterpret_cast<const uint4*>(expected + 32 * static_cast<int64_t>(i));
      const uint4 a0 = a[0], a1 = a[1], b0 = b[0], b1 = b[1];
      ok = (a0.x == b0.x && a0.y == b0.y && a0.z == b0.z && a0.w == b0.w && a1.x == b1.x &&
            a1.y == b1.y && a1.z == b1.z && a1.w == b1.w) ? 1 : 0;
    }
    scan[threadIdx.x] = ok;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {  // Hillis-Steele inclusive scan
      const int32_t v = threadIdx.x >= off ? scan[threadIdx.x - off] : 0;
      __syncthreads();
      scan[threadIdx.x] += v;
      __syncthreads();
    }
    if (ok) accepted[carry + scan[threadIdx.x] - 1] = payloads[i];
    carry += scan[255];
    __syncthreads();
  }
  if (threadIdx.x == 0) *count = carry;
}

}  // namespace p2p

using namespace p2p;

extern "C" int32_t p2p_sha256_batch(const uint8_t* const* msgs, const uint64_t* lens, int32_t k,
                                    uint8_t* digests, p2p_stream_t stream) {
  if (!msgs || !lens || !digests || k < 0) return P2P_ERR_INVALID;
  if (reinterpret_cast<uintptr_t>(digests) & 15) return P2P_ERR_ALIGN;
  if (k == 0) return P2P_OK;
  hipLaunchKernelGGL(sha256_pair_kernel, dim3((k + kShaLanes - 1) / kShaLanes), dim3(128), 0,
                     static_cast<hipStream_t>(stream), msgs, lens, k, digests);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? P2P_OK : static_cast<int32_t>(e);
}

extern "C" int32_t p2p_digest_accept(const uint8_t* digests, const uint8_t* expected,
                                     const float* const* payloads, int32_t k, const float** accepted,
                                     int32_t* count, p2p_stream_t stream) {
  if (!digests || !expected || !payloads || !accepted || !count || k < 0) return P2P_ERR_INVALID;
  if ((reinterpret_cast<uintptr_t>(digests) | reinterpret_cast<uintptr_t>(expected)) & 15)
    return P2P_ERR_ALIGN;
  hipLaunchKernelGGL(accept_kernel, dim3(1), dim3(256), 0, static_cast<hipStream_t>(stream), digests,
                     expected, payloads, k, accepted, count);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? P2P_OK : static_cast<int32_t>(e);
}
