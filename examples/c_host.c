/*
 * A host program in plain C over the C ABI (include/p2pdl.h) -- what a
 * non-Python host (cgo, JNI, N-API, ...) binds: device buffers from the HIP
 * runtime, a device array of peer pointers, one call per rule, results
 * checked against the same op sequences written here in C (reference
 * aggregator/aggregation.py:15-38 for FedAvg; the build-defined median of
 * include/p2pdl.h).  Built by p2pdl_amd/csrc/Makefile (gcc, no hipcc); run
 * by tests/test_c_host.py on a GPU.  Exit status 0 = every result bit-exact.
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/p2pdl.h"

#define HIP_OK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 2; } } while (0)
#define P2P_OK_(x) do { int32_t s_ = (x); if (s_ != P2P_OK) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, p2p_strerror(s_)); return 2; } } while (0)

enum { K = 7, N = 100003 };

static uint32_t lcg(uint32_t *s) { *s = *s * 1664525u + 1013904223u; return *s; }
static float uniform(uint32_t *s) { return (float)(lcg(s) >> 8) * 0x1p-24f * 2.0f - 1.0f; }

static uint32_t f2key(float f) {
  uint32_t b; memcpy(&b, &f, 4);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
static int cmp_key(const void *a, const void *b) {
  uint32_t x = f2key(*(const float *)a), y = f2key(*(const float *)b);
  return x < y ? -1 : x > y;
}

/* acc = +0; acc += peer in list order; acc / K (or * fl(1/K): torch on GPU
 * tensors); w + fl(lr * m), each op rounded. */
static void fedavg_ref(float *const *peers, const float *w0, float *w, int torch_gpu) {
  const float fk = (float)K, inv = 1.0f / fk;
  for (int i = 0; i < N; ++i) {
    float acc = 0.0f;
    for (int k = 0; k < K; ++k) acc = acc + peers[k][i];
    const float m = torch_gpu ? acc * inv : acc / fk;
    const float t = 0.1f * m;
    w[i] = w0[i] + t;
  }
}

static int compare(const char *what, const float *got, const float *want) {
  int bad = 0;
  for (int i = 0; i < N; ++i) bad += memcmp(&got[i], &want[i], 4) != 0;
  printf("%-26s %s (%d of %d differ)\n", what, bad ? "MISMATCH" : "bit-exact", bad, N);
  return bad;
}

int main(void) {
  if (p2p_abi_version() != P2P_ABI_VERSION) { fprintf(stderr, "ABI mismatch\n"); return 2; }
  uint32_t seed = 12345u;
  float *host[K], *dev[K], *w0 = malloc(4 * N), *got = malloc(4 * N), *want = malloc(4 * N);
  for (int k = 0; k < K; ++k) {
    host[k] = malloc(4 * N);
    for (int i = 0; i < N; ++i) host[k][i] = uniform(&seed) * 1e-2f;
    HIP_OK(hipMalloc((void **)&dev[k], 4 * N));
    HIP_OK(hipMemcpy(dev[k], host[k], 4 * N, hipMemcpyHostToDevice));
  }
  for (int i = 0; i < N; ++i) w0[i] = uniform(&seed) * 5e-2f;
  float **table, *w, *out;
  HIP_OK(hipMalloc((void **)&table, sizeof(float *) * K));  /* device array of device pointers */
  HIP_OK(hipMemcpy(table, dev, sizeof(float *) * K, hipMemcpyHostToDevice));
  HIP_OK(hipMalloc((void **)&w, 4 * N));
  HIP_OK(hipMalloc((void **)&out, 4 * N));
  hipStream_t stream;
  HIP_OK(hipStreamCreate(&stream));
  int bad = 0;

  /* FedAvg + apply, the reference's numerics (aggregation.py:15-38) */
  HIP_OK(hipMemcpy(w, w0, 4 * N, hipMemcpyHostToDevice));
  P2P_OK_(p2p_fedavg_apply_f32((const float *const *)table, K, N, w, 0.1f, stream));
  HIP_OK(hipStreamSynchronize(stream));
  HIP_OK(hipMemcpy(got, w, 4 * N, hipMemcpyDeviceToHost));
  fedavg_ref(host, w0, want, 0);
  bad += compare("fedavg", got, want);

  /* the same through the generic entry, torch's GPU division */
  HIP_OK(hipMemcpy(w, w0, 4 * N, hipMemcpyHostToDevice));
  P2P_OK_(p2p_aggregate_f32((const float *const *)table, K, N, P2P_RULE_FEDAVG_TORCH_GPU, 0, 0.1f, w, NULL,
                            stream));
  HIP_OK(hipStreamSynchronize(stream));
  HIP_OK(hipMemcpy(got, w, 4 * N, hipMemcpyDeviceToHost));
  fedavg_ref(host, w0, want, 1);
  bad += compare("fedavg_torch_gpu", got, want);

  /* coordinate-wise median, rank (K-1)/2 in the IEEE total order */
  P2P_OK_(p2p_median_f32((const float *const *)table, K, N, out, stream));
  HIP_OK(hipStreamSynchronize(stream));
  HIP_OK(hipMemcpy(got, out, 4 * N, hipMemcpyDeviceToHost));
  for (int i = 0; i < N; ++i) {
    float col[K];
    for (int k = 0; k < K; ++k) col[k] = host[k][i];
    qsort(col, K, 4, cmp_key);
    want[i] = col[(K - 1) / 2];
  }
  bad += compare("median", got, want);

  /* argument errors come back as codes, nothing launched */
  if (p2p_aggregate_f32((const float *const *)table, K, N, 4, 0, 0.1f, w, NULL, stream) != P2P_ERR_INVALID) {
    fprintf(stderr, "rule 4 accepted\n");
    ++bad;
  }
  HIP_OK(hipStreamDestroy(stream));
  for (int k = 0; k < K; ++k) { HIP_OK(hipFree(dev[k])); free(host[k]); }
  HIP_OK(hipFree(table)); HIP_OK(hipFree(w)); HIP_OK(hipFree(out));
  free(w0); free(got); free(want);
  return bad ? 1 : 0;
}
