#!/usr/bin/env python3
"""Same-process A/B (round 6, DESIGN §10 K1 open (b)): the chunk list of a
state_dict of separately allocated tensors (ops._chunk_plan, the split
kernel's chunks mode) as the product builds it -- eight 1024-float chunks
per tile, a partial last CU round -- against the same chunks spread over
whole CU rounds of tiles (ops.CHUNK_BALANCE_CUS: fewer chunks per tile, the
rest padding).  Cached launches timed by HIP events behind a spin,
alternated rep by rep; results bit-compared.  Measurement tool, not product.
usage: python tools/balance_ab.py [reps] [K:scale ...]   (default 64:1 16:1 32:1 64:2)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (the ResNet-18 shapes)
from p2pdl_amd import ops  # noqa: E402


def timed(fn, out):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(2_000_000)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    out.append(e0.elapsed_time(e1))


def one_case(K, scale, reps, dev, cus):
    sizes = [int(np.prod(s)) for _, s in bench.resnet18_param_shapes()] * scale
    nflat = sum(sizes)
    peers = [[torch.empty(n, dtype=torch.float32, device=dev) for n in sizes] for _ in range(K)]
    for p in range(K):
        for l, t in enumerate(peers[p]):
            ops.fill_synthetic_(t, 0x5EED0001 + l, p, 1e-2)
    w0 = [torch.empty(n, dtype=torch.float32, device=dev) for n in sizes]
    for l, w in enumerate(w0):
        ops.fill_synthetic_(w, 0x5EED0001 + l, 0xFFFFF, 5e-2)
    ptrs = np.array([[peers[p][l].data_ptr() for p in range(K)] for l in range(len(sizes))], dtype=np.uint64)
    legs = {"product (partial last round)": 0, f"balanced over {cus}-CU rounds": cus}
    res, ms, entries, wss = {}, {name: [] for name in legs}, {}, {}
    saved = ops.CHUNK_BALANCE_CUS
    try:
        for name, c in legs.items():
            ops.CHUNK_BALANCE_CUS = c
            ops._TABLES.clear()
            ops._LAYOUTS.clear()
            # each leg's w tensors stay alive as long as its cached entry is
            # relaunched: the entry holds their addresses (ops.relaunch's
            # contract -- a relaunch over freed w tensors writes into whatever
            # the allocator put there since, e.g. the other leg's table)
            wss[name] = [w.clone() for w in w0]
            ops.aggregate_ptr_table_(wss[name], ptrs, "fedavg")
            torch.cuda.synchronize()
            res[name] = torch.cat(wss[name]).cpu().numpy().view(np.uint32)
            entries[name] = next(reversed(ops._TABLES.values()))
        same = np.array_equal(*res.values())
        for _ in range(reps):
            for name in legs:
                e = entries[name]
                timed(lambda: ops.relaunch(e, dev, len(w0), K, 0.1), ms[name])
    finally:
        ops.CHUNK_BALANCE_CUS = saved
        ops._TABLES.clear()
        ops._LAYOUTS.clear()
    alg = 4.0 * nflat * (K + 2)
    tiles = {name: e[5][2][1] for name, e in entries.items()}
    print(f"K={K} x{scale}: {nflat:,} coords, tiles {tiles}, bit-identical: {same}")
    for name, v in ms.items():
        v = sorted(v)
        t = v[len(v) // 2]
        print(f"  {name:32s} median {t:.4f} ms  {alg / t / 1e6 / 8000:.4f} of 8 TB/s  best {v[0]:.4f}", flush=True)
    del peers
    torch.cuda.empty_cache()
    return same


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 21
    cases = [tuple(int(x) for x in a.split(":")) for a in sys.argv[2:]] or [(64, 1), (16, 1), (32, 1), (64, 2)]
    dev = torch.device("cuda", 0)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    ok = True
    for K, scale in cases:
        ok &= one_case(K, scale, reps, dev, cus)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
