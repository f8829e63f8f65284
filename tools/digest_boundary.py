"""Where the GPU SHA-256 batch kernel beats the host threads for host-resident
messages (utils/digests.py GPU_BATCH_MIN): digest_many over K distinct
messages of s bytes, cache cleared, host path (hashlib on the hashing
threads) vs GPU path (pack + one H2D + p2p_sha256_batch + D2H).  Writes one
JSON line per (K, s) and the crossover per size."""
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from p2pdl_amd.utils import digests  # noqa: E402


def timed(fn, reps=3):
    best = 1e9
    for _ in range(reps):
        digests.CACHE.clear()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    torch.cuda.init()
    rng = np.random.default_rng(1)
    rows = []
    for s in (64, 1024, 16384, 262144):
        for k in (64, 256, 1024, 4096, 16384):
            if k * s > (1 << 30):
                continue
            blob = rng.integers(0, 256, k * s, dtype=np.uint8).tobytes()
            msgs = [blob[i * s:(i + 1) * s] for i in range(k)]
            digests.GPU_BATCH_MIN = 1 << 62
            t_host = timed(lambda: digests.digest_many(msgs))
            digests.GPU_BATCH_MIN, digests.GPU_MAX_MESSAGE = 1, 1 << 62  # every batch to the GPU
            digests.digest_many(msgs)  # warm the kernel path
            t_gpu = timed(lambda: digests.digest_many(msgs))
            digests.CACHE.clear()
            got = digests.digest_many(msgs)
            assert got[0] == hashlib.sha256(msgs[0]).digest() and got[-1] == hashlib.sha256(msgs[-1]).digest()
            row = {"k": k, "bytes": s, "host_ms": round(t_host * 1e3, 3), "gpu_ms": round(t_gpu * 1e3, 3),
                   "gpu_wins": t_gpu < t_host, "threads": digests.hash_pool()._max_workers}
            rows.append(row)
            print(json.dumps(row), flush=True)
    cross = {}
    for s in sorted({r["bytes"] for r in rows}):
        ks = [r["k"] for r in rows if r["bytes"] == s and r["gpu_wins"]]
        cross[s] = min(ks) if ks else None
    print(json.dumps({"crossover_k_by_bytes": cross}), flush=True)
    if out:
        with open(out, "w") as f:
            json.dump({"rows": rows, "crossover_k_by_bytes": cross}, f, indent=1)


if __name__ == "__main__":
    main()
