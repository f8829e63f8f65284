#!/usr/bin/env python3
"""Same-box A/B (round 5): a ResNet-18 state_dict x 64 updates (cfg2) through
the segment path with the split plan (LDS-DMA split kernel over whole tiles +
the VGPR segment kernel over the rest) against the VGPR segment kernel alone
(ops._split_plan forced off), interleaved, HIP events; results bit-compared.
Measurement tool, not product.  usage: python tools/seg_ab.py [reps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (the ResNet-18 shapes)
from p2pdl_amd import ops  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    K = 64
    shapes = bench.resnet18_param_shapes()
    sizes = [int(np.prod(s)) for _, s in shapes]
    offs, o = [], 0
    for n in sizes:
        offs.append(o)
        o += -(-n // 64) * 64
    slab = torch.empty((K, o), dtype=torch.float32, device=dev)
    for p in range(K):
        ops.fill_synthetic_(slab[p], 0x5EED0001, p, 1e-2)
    w0 = [torch.empty(n, dtype=torch.float32, device=dev) for n in sizes]
    for i, w in enumerate(w0):
        ops.fill_synthetic_(w, 0x5EED0001 + i, 0xFFFFF, 5e-2)
    real = ops._split_plan
    variants = {"split+segments": real, "segments only": lambda *a, **k: None}
    res = {}
    for name, plan in variants.items():
        ops._split_plan = plan
        ops._TABLES.clear()
        ws = [w.clone() for w in w0]
        ops.aggregate_slab_rows_(ws, slab, list(range(K)), offs, "fedavg")
        torch.cuda.synchronize()
        res[name] = torch.cat(ws).cpu().numpy()
    ops._split_plan = real
    same = np.array_equal(res["split+segments"].view(np.uint32), res["segments only"].view(np.uint32))
    print(f"bit-identical: {same}")
    ms = {k: [] for k in variants}
    ws = [w.clone() for w in w0]
    for _ in range(reps):
        for name, plan in variants.items():
            ops._split_plan = plan
            ops._TABLES.clear()
            ops.aggregate_slab_rows_(ws, slab, list(range(K)), offs, "fedavg")  # builds + caches the table
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(2_000_000)
            e0.record()
            ops.aggregate_slab_rows_(ws, slab, list(range(K)), offs, "fedavg")  # cached: the launches only
            e1.record()
            torch.cuda.synchronize()
            ms[name].append(e0.elapsed_time(e1))
    ops._split_plan = real
    alg = 4.0 * sum(sizes) * (K + 2)
    for name, v in ms.items():
        v = sorted(v)
        t = v[len(v) // 2]
        print(f"{name:16s} median {t:.4f} ms  {alg / t / 1e9:.1f} GB/s  {alg / t / 1e9 / 8000:.4f} of 8 TB/s  best {v[0]:.4f}")
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
