#!/usr/bin/env python3
"""Lab (round 5): the VGPR FedAvg kernels' aligned paths under one library
build (P2P_LIB): the segment kernel over ResNet-18's 62 tensors x 64 updates
as separate tensors (the drop-in's general path), the flat kernel at K = 4 x
100M and K = 8 x 30M (below the split kernel's K), and 4-B aligned rows
(the element-wise path).  Prints one line per case.  usage: P2P_LIB=... python tools/vgpr_ab.py [reps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from p2pdl_amd import ops  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    v = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(1_000_000)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        v.append(e0.elapsed_time(e1))
    return sorted(v)[len(v) // 2]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 15
    dev = torch.device("cuda", 0)
    lib = os.path.basename(os.environ.get("P2P_LIB", "product"))
    sizes = [int(np.prod(s)) for _, s in bench.resnet18_param_shapes()]
    K = 64
    peers = [[torch.empty(n, device=dev) for n in sizes] for _ in range(K)]
    for j in range(K):
        for i, t in enumerate(peers[j]):
            ops.fill_synthetic_(t, 5 + i, j, 1e-2)
    ws = [torch.zeros(n, device=dev) for n in sizes]
    t = timeit(lambda: ops.aggregate_segments_(ws, peers, "fedavg"), reps)
    print(f"{lib} segments cfg2 general path: {t:.4f} ms {4.0 * sum(sizes) * (K + 2) / t / 1e6 / 8000:.4f}")
    del peers
    for k, n, off in ((4, 100_000_000, 0), (8, 30_000_000, 0), (8, 30_000_000, 1)):
        slab = torch.empty(k * (n + 64) + 8, device=dev)
        rows = [slab[off + j * (n + 64): off + j * (n + 64) + n] for j in range(k)]
        for j, r in enumerate(rows):
            ops.fill_synthetic_(r, 9, j, 1e-2)
        w = torch.zeros(n, device=dev)
        t = timeit(lambda: ops.aggregate(rows, "fedavg", w=w), reps)
        print(f"{lib} flat K={k} n={n:,} offset {off}: {t:.4f} ms {4.0 * n * (k + 2) / t / 1e6 / 8000:.4f}")
        del slab


if __name__ == "__main__":
    main()
