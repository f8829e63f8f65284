#!/usr/bin/env python3
"""Same-box A/B (round 5): cfg2 -- ResNet-18's 62 tensors x 64 updates in a
DeviceInbox slab (chunk layout) -- FedAvg through the rows kernel (the slab
rows as flat peers, ops._rows_entry) against the VGPR segment kernel over
the same rows (the rows entry forced off), interleaved, HIP events,
bit-compared.  Measurement tool, not product.  usage: python tools/rows_ab.py [reps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (the ResNet-18 shapes)
from p2pdl_amd import ops  # noqa: E402
from p2pdl_amd.node.inbox import DeviceInbox  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    K = 64
    shapes = bench.resnet18_param_shapes()
    template = {name: torch.zeros(s, device=dev) for name, s in shapes}
    inbox = DeviceInbox(template, k_max=K, device=dev)
    offs = [inbox.layout[name][0] for name, _ in shapes]
    sizes = [int(np.prod(s)) for _, s in shapes]
    print(f"row {inbox.row:,} floats for {sum(sizes):,} parameters; chunk layout: {all(o % 1024 == 0 for o in offs)}")
    for p in range(K):
        ops.fill_synthetic_(inbox.slab[p], 0x5EED0001, p, 1e-2)
    w0 = [torch.empty(n, dtype=torch.float32, device=dev) for n in sizes]
    for i, w in enumerate(w0):
        ops.fill_synthetic_(w, 0x5EED0001 + i, 0xFFFFF, 5e-2)
    real = ops._rows_entry
    variants = {"rows kernel": real, "segment kernel": lambda *a, **k: None}
    res = {}
    try:
        for name, fn in variants.items():
            ops._rows_entry = fn
            ops._TABLES.clear()
            ws = [w.clone() for w in w0]
            ops.aggregate_slab_rows_(ws, inbox.slab, list(range(K)), offs, "fedavg")
            torch.cuda.synchronize()
            res[name] = torch.cat(ws).cpu().numpy()
        same = np.array_equal(res["rows kernel"].view(np.uint32), res["segment kernel"].view(np.uint32))
        ms = {k: [] for k in variants}
        ws = [w.clone() for w in w0]
        for _ in range(reps):
            for name, fn in variants.items():
                ops._rows_entry = fn
                ops._TABLES.clear()
                ops.aggregate_slab_rows_(ws, inbox.slab, list(range(K)), offs, "fedavg")  # builds + caches
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda._sleep(2_000_000)
                e0.record()
                ops.aggregate_slab_rows_(ws, inbox.slab, list(range(K)), offs, "fedavg")  # cached: the launch
                e1.record()
                torch.cuda.synchronize()
                ms[name].append(e0.elapsed_time(e1))
    finally:
        ops._rows_entry = real
    alg = 4.0 * sum(sizes) * (K + 2)
    print(f"bit-identical: {same}")
    for name, v in ms.items():
        v = sorted(v)
        t = v[len(v) // 2]
        print(f"  {name:16s} median {t:.4f} ms  {alg / t / 1e6 / 8000:.4f} of 8 TB/s  best {v[0]:.4f}")
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
