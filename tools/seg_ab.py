#!/usr/bin/env python3
"""Same-box A/B (round 5): a state_dict of ResNet-18's shapes (cfg2), and the
same shapes repeated `scale` times, x 64 updates through the segment path
with the split plan (LDS-DMA split kernel over whole tiles + the VGPR segment
kernel over the rest) against the VGPR segment kernel alone (ops._split_plan
forced off), interleaved, HIP events; results bit-compared.  Then the same
bytes as one flat buffer per peer (split rounds + the VGPR kernel's rest).
Measurement tool, not product.  usage: python tools/seg_ab.py [reps] [scale ...]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (the ResNet-18 shapes)
from p2pdl_amd import ops  # noqa: E402

K = 64


def timed(fn, reps_out, dev):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(2_000_000)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize(dev)
    reps_out.append(e0.elapsed_time(e1))


def one_scale(scale, reps, dev):
    sizes = [int(np.prod(s)) for _, s in bench.resnet18_param_shapes()] * scale
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
    try:
        for name, plan in variants.items():
            ops._split_plan = plan
            ops._TABLES.clear()
            ws = [w.clone() for w in w0]
            ops.aggregate_slab_rows_(ws, slab, list(range(K)), offs, "fedavg")
            torch.cuda.synchronize()
            res[name] = torch.cat(ws).cpu().numpy()
        same = np.array_equal(res["split+segments"].view(np.uint32), res["segments only"].view(np.uint32))
        ms = {k: [] for k in variants}
        ws = [w.clone() for w in w0]
        for _ in range(reps):
            for name, plan in variants.items():
                ops._split_plan = plan
                ops._TABLES.clear()
                ops.aggregate_slab_rows_(ws, slab, list(range(K)), offs, "fedavg")  # builds + caches the table
                timed(lambda: ops.aggregate_slab_rows_(ws, slab, list(range(K)), offs, "fedavg"), ms[name], dev)
    finally:
        ops._split_plan = real
    nflat = sum(sizes)
    table = ops.pointer_table([slab[p, :nflat] for p in range(K)], dev)
    wf = torch.empty(nflat, dtype=torch.float32, device=dev)
    ops.fill_synthetic_(wf, 0x5EED0001, 0xFFFFF, 5e-2)
    ms["flat (same bytes)"] = []
    for _ in range(reps):
        timed(lambda: ops.aggregate(None, "fedavg", w=wf, lr=0.1, table=table), ms["flat (same bytes)"], dev)
    alg = 4.0 * nflat * (K + 2)
    print(f"x{scale}: {len(sizes)} tensors, {nflat:,} coords, bit-identical: {same}")
    for name, v in ms.items():
        v = sorted(v)
        t = v[len(v) // 2]
        print(f"  {name:18s} median {t:.4f} ms  {alg / t / 1e6:.1f} GB/s  {alg / t / 1e6 / 8000:.4f} of 8 TB/s  "
              f"best {v[0]:.4f}")
    return same


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    scales = [int(a) for a in sys.argv[2:]] or [1]
    dev = torch.device("cuda", 0)
    ok = True
    for s in scales:
        ok &= one_scale(s, reps, dev)
        torch.cuda.empty_cache()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
