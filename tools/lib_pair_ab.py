#!/usr/bin/env python3
"""Same-process A/B of the product library against other builds (round 6).

Bench-level A/Bs that alternate processes carried an order effect on these
boxes: whichever build ran first in a round read 2-3% faster, whatever it was
(profiles/r06/queue_ab/README.md).  Here every build is loaded into ONE
process (ctypes, the same ABI), the same device buffers are reduced by each
in turn, rep by rep, each launch queued behind a spin kernel and timed with
HIP events; the builds' outputs are bit-compared.  Flat FedAvg
(p2p_aggregate_f32), one launch per case -- the cfg3 plane shapes and others.
Measurement tool, not product.
usage: python tools/lib_pair_ab.py <reps> <tag> [<tag> ...] -- <K:n> ...
  tag "prod" = p2pdl_amd/libp2pdl_hip.so, tag X = tools/libp2pdl_X.so"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from p2pdl_amd import _native as N  # noqa: E402
from p2pdl_amd import ops  # noqa: E402


def load(tag):
    path = N.LIB_PATH if tag == "prod" else os.path.join(REPO, "tools", f"libp2pdl_{tag}.so")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    f = lib.p2p_aggregate_f32
    f.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_float,
                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    f.restype = ctypes.c_int32
    return f


def main():
    i = sys.argv.index("--")
    reps, tags = int(sys.argv[1]), sys.argv[2:i]
    cases = [tuple(int(x) for x in c.split(":")) for c in sys.argv[i + 1:]]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    fns = {t: load(t) for t in tags}
    ok = True
    for K, n in cases:
        pitch = -(-n // 64) * 64
        slab = torch.empty((K, pitch), dtype=torch.float32, device=dev)
        for p in range(K):
            ops.fill_synthetic_(slab[p, :n], 0x5EED0002, p, 1e-2)
        table = ops.pointer_table([slab[p, :n] for p in range(K)], dev)
        w0 = torch.empty(n, dtype=torch.float32, device=dev)
        ops.fill_synthetic_(w0, 0x5EED0002, 0xFFFFF, 5e-2)
        outs = {}
        st = torch.cuda.current_stream(dev).cuda_stream
        for t, f in fns.items():
            w = w0.clone()
            assert f(table.data_ptr(), K, n, 0, 0, 0.1, w.data_ptr(), None, st) == 0
            torch.cuda.synchronize()
            outs[t] = w.cpu().numpy().view(np.uint32)
        same = all(np.array_equal(outs[t], outs[tags[0]]) for t in tags)
        ok &= same
        w = w0.clone()
        ms = {t: [] for t in tags}
        for r in range(reps):
            order = tags if r % 2 == 0 else tags[::-1]
            for t in order:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda._sleep(2_000_000)
                e0.record()
                fns[t](table.data_ptr(), K, n, 0, 0, 0.1, w.data_ptr(), None, st)
                e1.record()
                torch.cuda.synchronize()
                ms[t].append(e0.elapsed_time(e1))
        alg = 4.0 * n * (K + 2)
        print(f"K={K} n={n:,}  bit-identical across builds: {same}")
        for t, v in ms.items():
            v = sorted(v)
            med = v[len(v) // 2]
            print(f"  {t:10s} median {med:.4f} ms  {alg / med / 1e6 / 8000:.4f} of 8 TB/s  best {alg / v[0] / 1e6 / 8000:.4f}"
                  f"  worst {alg / v[-1] / 1e6 / 8000:.4f}", flush=True)
        del slab, table, w0, w
        torch.cuda.empty_cache()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
