/*
 * p2pdl.h -- C ABI of the MI355X (gfx950) aggregation / digest hot path.
 *
 * Drop-in boundary for P2PDL's data-parallel hot path.
 * Plain pointers and sizes only: no torch / C++ types cross this ABI.  The
 * Python host layer (p2pdl_amd/_native.py) binds these with ctypes; the
 * binding a maintainer would add to the reference is in INTEGRATION.md.
 *
 * Conventions
 *   - Every pointer named peers / w / out / msgs / lens / digests is a DEVICE
 *     pointer.  `peers` is a device array of K device pointers, one per peer
 *     update, in the order of the reference's received_models list
 *     (reference node/node.py:141 appends in arrival order; the reference
 *     sums in that order, aggregator/aggregation.py:25).
 *   - `stream` is a hipStream_t (NULL = legacy default stream).  All calls are
 *     asynchronous, stream-ordered, allocate nothing and keep no state
 *     (re-entrant; safe inside hipGraph capture).
 *   - Return value: 0 = OK; < 0 = library error (P2P_ERR_*); > 0 = the
 *     hipError_t of a failed launch.  p2p_strerror() describes any code.
 *     No exception ever crosses the ABI.
 *   - Numerics are bit-exact to the reference CPU op sequence:
 *     +0 accumulator init, fixed peer order, IEEE true division by K, and
 *     w + lr*agg with the multiply and the add separately rounded (no FMA);
 *     P2P_RULE_FEDAVG_TORCH_GPU divides as torch does on GPU tensors.
 */
#ifndef P2PDL_H
#define P2PDL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: p2p_set_robust_layout (a process-global A/B switch of version 1) is
 *    gone; every other entry point is unchanged.
 * 3: adds p2p_land_segments_f32 (K5, landing a received update).
 * 4: adds the rule P2P_RULE_FEDAVG_TORCH_GPU and p2p_fedavg_apply_16
 *    (float16 / bfloat16 models).
 * 5: P2P_DELTA_TILE 4096 -> 1024 (the delta segment table's tile_begin is
 *    counted in 1024-element tiles).
 * 6: adds p2p_fedavg_split_plan / p2p_fedavg_split_segments_f32 (whole
 *    tiles of a state_dict on the LDS-DMA split kernel).
 * 7: adds p2p_fedavg_split_rows_f32 / p2p_row_chunk_t (a state_dict slab's
 *    rows as flat peers, the model scattered by 1024-float chunks).
 * 8: adds p2p_fedavg_split_chunks_f32 (a state_dict of separately allocated
 *    tensors on the split kernel, one launch, by 1024-float chunks).
 * 9: adds p2p_aggregate_ex_f32 and P2P_HINT_SHARE_CUS (the FedAvg split
 *    kernel's tile queue vs a kernel running beside it). */
#define P2P_ABI_VERSION 9

typedef void *p2p_stream_t; /* hipStream_t */

enum {
  P2P_OK = 0,
  P2P_ERR_INVALID = -1,     /* bad argument (null pointer, k < 1, n < 0, bad trim) */
  P2P_ERR_UNSUPPORTED = -2, /* valid but unsupported here (robust rules need k <= 256) */
  P2P_ERR_ALIGN = -3        /* a float pointer that is not 4-byte aligned */
};

/* P2P_RULE_FEDAVG: the reference's ops as torch runs them on CPU tensors
 * (acc / K, IEEE division; the committed golden vectors).
 * P2P_RULE_FEDAVG_TORCH_GPU: the same ops as torch runs them on GPU tensors,
 * the reference's own deployment (node/node.py:28-29 puts the model on
 * cuda): ATen divides by the CPU scalar K as acc * fl(1/K) (ABI 4). */
enum { P2P_RULE_FEDAVG = 0, P2P_RULE_MEDIAN = 1, P2P_RULE_TRIMMED = 2, P2P_RULE_FEDAVG_TORCH_GPU = 3 };

/* One tensor of a state_dict (reference: one key of self.model.state_dict(),
 * aggregator/aggregation.py:15,27,37).  Device-resident table entry. */
typedef struct p2p_segment_t {
  const float *const *peers; /* device array of K device pointers: this key of each update */
  float *w;                  /* model tensor for this key, updated in place (nullable) */
  float *out;                /* receives the aggregate before apply (nullable) */
  int64_t n;                 /* elements in this tensor */
  int64_t tile_begin;        /* sum of ceil(n_j / p2p_tile_elems(rule, k)) over earlier segments */
} p2p_segment_t;

/* ABI version (P2P_ABI_VERSION) and error text (static storage). */
int32_t p2p_abi_version(void);
const char *p2p_strerror(int32_t code);

/* Elements per tile of the segment kernel for `rule` with k peers (host
 * planning helper for p2p_segment_t.tile_begin).  A pure function of
 * (rule, k): FedAvg 4096; median / trimmed 128 for k <= 128, 64 for
 * k in 129..256. */
int64_t p2p_tile_elems(int32_t rule, int32_t k);

/* ---- K1: FedAvg --------------------------------------------------------
 * Replaces reference aggregator/aggregation.py:15-38 for one flat buffer:
 *   acc = +0 (:15); acc += peers[j] for j in list order (:25-28);
 *   acc /= K (:31-32); w += fp32(lr) * acc (:36-38, lr = 0.1 there).
 * Kernel choice (a pure function of k and n, same bits either way): for
 * 16 <= k <= 128, every whole 8192-float tile (from one round of the CU
 * count up) runs on the LDS-DMA split kernel (loader + consumer waves; a
 * persistent grid of one block per CU claiming tiles from a counter pair of
 * a device-global ring, which each launch leaves zeroed), the < 8192-float
 * tail on the VGPR kernel; for 129 <= k <= 256 whole rounds of tiles run on
 * the same queued kernel, the rest on the VGPR kernel; above 256, under
 * P2P_HINT_SHARE_CUS (p2p_aggregate_ex_f32) and on the device-K path the
 * split kernel runs one block per tile over whole rounds of tiles and the
 * VGPR kernel the rest.  The peer pointers
 * are read from device memory each launch; 4-byte-aligned (not 16-byte)
 * pointers are handled, more slowly. */
int32_t p2p_fedavg_apply_f32(const float *const *peers, int32_t k, int64_t n, float *w, float lr,
                             p2p_stream_t stream);
/* Same reduction, writes acc/K to out (the :15-32 part, no apply). */
int32_t p2p_mean_f32(const float *const *peers, int32_t k, int64_t n, float *out,
                     p2p_stream_t stream);
/* FedAvg over a device-resident peer count: K = *k_dev (1 <= K <= k_max),
 * peers[0..K-1] used.  Feeds the fused digest -> accept -> FedAvg path. */
int32_t p2p_fedavg_apply_devk_f32(const float *const *peers, const int32_t *k_dev, int32_t k_max,
                                  int64_t n, float *w, float lr, float *out, p2p_stream_t stream);

/* ---- K2: robust rules (build-defined: reference README.md:10 TODO) -----
 * median: rank (K-1)/2 under the IEEE total order on float bits.
 * trimmed: ascending fp32 sum of sorted ranks b..K-b-1 from +0, / (K-2b).
 * k <= 256.  Kernel family (a pure function of (rule, k, trim_b); no process
 * state): one lane per coordinate for k <= 128; for k = 256 with the median
 * or the default trim (b = 51) one lane per coordinate in two-wave blocks,
 * each wave holding 128 peers (robust_pair.hip); for every other k in
 * 129..256 (or trim) 4 lanes x 64 keys per coordinate, peer rows LDS-DMA
 * staged (robust_lds.hip). */
int32_t p2p_median_f32(const float *const *peers, int32_t k, int64_t n, float *out,
                       p2p_stream_t stream);
int32_t p2p_trimmed_mean_f32(const float *const *peers, int32_t k, int64_t n, int32_t trim_b,
                             float *out, p2p_stream_t stream);

/* Generic fused form of K1/K2: rule in P2P_RULE_*; writes the aggregate to
 * out (nullable) and applies w += lr*agg when w is non-null (at least one of
 * w, out must be non-null).  trim_b is read only for P2P_RULE_TRIMMED. */
int32_t p2p_aggregate_f32(const float *const *peers, int32_t k, int64_t n, int32_t rule,
                          int32_t trim_b, float lr, float *w, float *out, p2p_stream_t stream);

/* p2p_aggregate_f32 with launch hints (0 = p2p_aggregate_f32).
 * P2P_HINT_SHARE_CUS: another kernel runs beside this call on another stream
 * -- the all-gather of a sharded round (p2pdl_amd/sharded.py PeerPlanes,
 * SURVEY.md §8(e)).  The FedAvg split kernel then runs one block per tile,
 * so each tile's end frees a CU the dispatcher can hand to that kernel,
 * instead of its persistent tile-queue grid (8 <= k <= 256), which holds
 * every CU until the launch ends.  Same results either way; unknown hint bits are
 * P2P_ERR_INVALID. */
#define P2P_HINT_SHARE_CUS 1
int32_t p2p_aggregate_ex_f32(const float *const *peers, int32_t k, int64_t n, int32_t rule, int32_t trim_b,
                             float lr, float *w, float *out, int32_t hints, p2p_stream_t stream);

/* The LDS-DMA split kernel over whole P2P_SPLIT_TILE-element tiles of a
 * segment table (FedAvg rules only): entry t of the DEVICE array `tiles`
 * names segment `seg` of `segs` and the tile's first element `c0` in it.
 * Precondition (the caller's, checked where the list is built): every listed
 * segment's K peer pointers and w / out are 16-byte aligned and
 * c0 + P2P_SPLIT_TILE <= n.  The rest of each segment goes through
 * p2p_aggregate_segments_f32 (a table of the remaining ranges).
 * p2p_fedavg_split_plan(k, full) is how many of `full` whole tiles to list:
 * whole rounds of the device's CU count, 0 for k < 16 (same results either
 * way; the plan is speed only). */
#define P2P_SPLIT_TILE 8192
typedef struct p2p_split_tile_t {
  int64_t seg; /* index into segs */
  int64_t c0;  /* first element of the tile inside the segment */
} p2p_split_tile_t;
int64_t p2p_fedavg_split_plan(int32_t k, int64_t full_tiles);
int32_t p2p_fedavg_split_segments_f32(const p2p_split_tile_t *tiles, int64_t ntiles, const p2p_segment_t *segs,
                                      int32_t k, int32_t rule, float lr, p2p_stream_t stream);

/* FedAvg over the K rows of a state_dict slab (node/inbox.py DeviceInbox) on
 * the split kernel, one launch, every tile whole: `rows` is a DEVICE array of
 * K row pointers (16-B aligned) each holding ntiles * P2P_SPLIT_TILE floats;
 * chunks[c] (DEVICE, ntiles * 8 entries) is the model tensor memory the
 * row's floats [P2P_ROW_CHUNK * c, + P2P_ROW_CHUNK) update -- `w` 16-B
 * aligned, `valid` how many of the chunk's floats it holds (<= 1024, 0 or w
 * NULL for padding between keys, which is averaged and dropped).  The
 * model's keys must therefore start on P2P_ROW_CHUNK boundaries of the row.
 * w[i] += lr * mean_k(row_k[c0 + i]) with the same per-element op order as
 * p2p_fedavg_apply_f32 (FedAvg rules only). */
#define P2P_ROW_CHUNK 1024
typedef struct {
  float *w;
  int64_t valid;
} p2p_row_chunk_t;
int32_t p2p_fedavg_split_rows_f32(const float *const *rows, int32_t k, int64_t ntiles, const p2p_row_chunk_t *chunks,
                                  int32_t rule, float lr, p2p_stream_t stream);

/* FedAvg over a whole state_dict of separately allocated tensors -- what the
 * reference's receive path hands aggregate_models (node/node.py:138-141
 * pickle.loads, aggregator/aggregation.py:25-38) -- on the split kernel in
 * ONE launch.  `chunks` (DEVICE, ntiles * 8 entries) lists P2P_ROW_CHUNK-
 * element chunks of the segments of `segs`: entry c names segment `seg` (-1:
 * padding, no work) and the chunk's first element `c0` (a multiple of 4) in
 * it; the chunk covers elements [c0, c0 + min(P2P_ROW_CHUNK, n - c0)).
 * Split tile t is chunks 8t .. 8t + 7.  Every listed segment's K peer
 * pointers and w / out must be 16-byte aligned (the caller's check); a
 * segment's tile_begin is not read.  No read leaves a segment's tensors.
 * Same per-element op order as p2p_fedavg_apply_f32 (FedAvg rules only).
 * ABI 8. */
int32_t p2p_fedavg_split_chunks_f32(const p2p_split_tile_t *chunks, int64_t ntiles, const p2p_segment_t *segs,
                                    int32_t k, int32_t rule, float lr, p2p_stream_t stream);

/* Whole state_dict in ONE launch: segs is a DEVICE array of nseg entries
 * (tile_begin prefix-summed with p2p_tile_elems(rule, k)); total_tiles is the
 * sum over all segments.  Replaces the per-key loops of
 * aggregator/aggregation.py:15,25-28,31-32,37-38. */
int32_t p2p_aggregate_segments_f32(const p2p_segment_t *segs, int32_t nseg, int64_t total_tiles,
                                   int32_t k, int32_t rule, int32_t trim_b, float lr,
                                   p2p_stream_t stream);

/* FedAvg + apply on a float16 / bfloat16 model (aggregation.py:15-38 on a
 * half-precision state_dict): peers / w hold the 16-bit storage of `dtype`
 * (P2P_DTYPE_F16 or P2P_DTYPE_BF16); every op computed in fp32 and rounded
 * to the storage type, as torch runs the reference's ops -- acc = r(acc + u)
 * per update in list order, r(acc / K) (P2P_RULE_FEDAVG) or r(acc * fl(1/K))
 * (P2P_RULE_FEDAVG_TORCH_GPU), w = r(w + r(lr * acc)). */
enum { P2P_DTYPE_F16 = 1, P2P_DTYPE_BF16 = 2 };
int32_t p2p_fedavg_apply_16(const uint16_t *const *peers, int32_t k, int64_t n, uint16_t *w, float lr,
                            int32_t dtype, int32_t rule, p2p_stream_t stream);

/* w += lr * agg, multiply and add separately rounded (aggregation.py:36-38). */
int32_t p2p_apply_f32(float *w, const float *agg, float lr, int64_t n, p2p_stream_t stream);

/* ---- K4: trainer-side local update ---------------
 * Replaces reference node/node.py:273-282: delta = current - previous
 * (:278-279), then previous = current (the clone at :282).  first != 0 is
 * the first round (previous is None, :272-275): delta = current.  One pass,
 * 16 bytes of HBM traffic per coordinate; fp32 subtraction is IEEE exact. */
int32_t p2p_delta_snapshot_f32(const float *cur, float *prev, float *delta, int64_t n, int32_t first,
                               p2p_stream_t stream);

#define P2P_DELTA_TILE 1024 /* elements per tile of the delta segment kernel */

/* One tensor of a state_dict for the delta kernel (device-resident entry). */
typedef struct p2p_delta_segment_t {
  const float *cur; /* current parameter (model.state_dict()[key]) */
  float *prev;      /* previous snapshot, overwritten with cur */
  float *delta;     /* receives cur - prev */
  int64_t n;
  int64_t tile_begin; /* sum of ceil(n_j / P2P_DELTA_TILE) over earlier segments */
} p2p_delta_segment_t;

/* Whole state_dict in one launch (segs is a DEVICE array). */
int32_t p2p_delta_snapshot_segments_f32(const p2p_delta_segment_t *segs, int32_t nseg, int64_t total_tiles,
                                        int32_t first, p2p_stream_t stream);

/* ---- K5: landing a received update ---------------
 * Replaces the per-tensor unpickling of reference node/node.py:135-141 for the
 * fp32 payloads of one serialized update: msg is the whole message, copied
 * to the device as bytes (msg_bytes of them); segment j copies n fp32 values
 * from byte offset src_off of msg (any alignment) to dst (4-B aligned, e.g.
 * a tensor's offset in its slab row).  Reads stay below msg_bytes. */
#define P2P_LAND_TILE 4096 /* fp32 values per tile of the landing kernel */

typedef struct p2p_land_segment_t {
  uint64_t src_off;   /* byte offset of the payload in msg */
  float *dst;         /* destination of n fp32 values */
  int64_t n;
  int64_t tile_begin; /* sum of ceil(n_j / P2P_LAND_TILE) over earlier segments */
} p2p_land_segment_t;

/* One launch per update (segs is a DEVICE array of nseg entries). */
int32_t p2p_land_segments_f32(const uint8_t *msg, uint64_t msg_bytes, const p2p_land_segment_t *segs,
                              int32_t nseg, int64_t total_tiles, p2p_stream_t stream);

/* ---- K3: SHA-256 over serialized updates --------------------------------
 * digests[32*i .. 32*i+31] = SHA-256(msgs[i][0 .. lens[i]-1]) (FIPS 180-4),
 * the digest inside ECDSA(SHA256()) of reference utils/crypto.py:54-57 (sign)
 * and :92-96 (verify).  msgs, lens, digests are device arrays. */
int32_t p2p_sha256_batch(const uint8_t *const *msgs, const uint64_t *lens, int32_t k,
                         uint8_t *digests, p2p_stream_t stream);

/* Accept step of the fused path: keeps peer i iff digests[i] == expected[i]
 * (32 bytes each); writes the kept payload pointers, in the original list
 * order, to accepted[0..count-1] and count to *count (both device). */
int32_t p2p_digest_accept(const uint8_t *digests, const uint8_t *expected,
                          const float *const *payloads, int32_t k, const float **accepted,
                          int32_t *count, p2p_stream_t stream);

/* ---- synthetic inputs ---------------------------------
 * out[i] = ((splitmix64(seed ^ (peer << 40) ^ g(i)) >> 40) * 2^-23 - 1) * scale
 * with g(i) the global coordinate of local element i under round-robin chunk
 * ownership (chunk elements per chunk; g(i) = i when nranks <= 1). */
int32_t p2p_fill_synthetic_f32(float *out, int64_t n, uint64_t seed, int32_t peer, float scale,
                               int64_t chunk, int32_t nranks, int32_t rank, p2p_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* P2PDL_H */
