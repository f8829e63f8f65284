#!/usr/bin/env python3
"""Same-box A/B (round 6): a state_dict of separately
allocated tensors -- what pickle.loads hands the reference's listener
(node/node.py:138-141) -- x K updates through each ops.STATE_DICT_ROUTE:

  chunks  one split launch by 1024-float chunks (p2p_fedavg_split_chunks_f32)
  tiles   round 5's whole-tile split plan (gate off) + the VGPR kernel's rest
  vgpr    the VGPR segment kernel alone (round 5's product below 2048 tiles)

and, for reference, the same model landed in a DeviceInbox slab (the rows
kernel) and the same bytes as one flat buffer per peer.  Interleaved, HIP
events around the cached launch (ops.aggregate_ptr_table_'s table built
first), results bit-compared across routes; then host wall time per call
with a fresh table every call (the host's chunk-list build + H2D).
Measurement tool, not product.
usage: python tools/chunks_ab.py [reps] [K:scale ...]   (default 64:1 16:1 64:4)"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (the ResNet-18 shapes)
from p2pdl_amd import ops  # noqa: E402

ROUTES = ("chunks", "tiles", "vgpr")


def timed(fn, out, dev):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(2_000_000)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize(dev)
    out.append(e0.elapsed_time(e1))


def one_case(K, scale, reps, dev):
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
    saved = (ops.STATE_DICT_ROUTE, ops.SPLIT_SEGMENT_MIN_TILES)
    res, ms, fresh = {}, {r: [] for r in ROUTES}, {}
    try:
        ops.SPLIT_SEGMENT_MIN_TILES = 0
        for r in ROUTES:
            ops.STATE_DICT_ROUTE = r
            ops._TABLES.clear()
            ws = [w.clone() for w in w0]
            ops.aggregate_ptr_table_(ws, ptrs, "fedavg")
            torch.cuda.synchronize()
            res[r] = torch.cat(ws).cpu().numpy().view(np.uint32)
        same = all(np.array_equal(res[r], res["vgpr"]) for r in ROUTES)
        ws = [w.clone() for w in w0]
        for _ in range(reps):
            for r in ROUTES:
                ops.STATE_DICT_ROUTE = r
                ops._TABLES.clear()
                ops.aggregate_ptr_table_(ws, ptrs, "fedavg")  # builds + caches the table
                timed(lambda: ops.aggregate_ptr_table_(ws, ptrs, "fedavg"), ms[r], dev)
        for r in ("chunks", "vgpr"):  # host wall time per call, a new table every call
            ops.STATE_DICT_ROUTE = r
            t = []
            for _ in range(reps):
                ops._TABLES.clear()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ops.aggregate_ptr_table_(ws, ptrs, "fedavg")
                torch.cuda.synchronize()
                t.append(time.perf_counter() - t0)
            fresh[r] = sorted(t)[len(t) // 2] * 1e3
    finally:
        ops.STATE_DICT_ROUTE, ops.SPLIT_SEGMENT_MIN_TILES = saved
        ops._TABLES.clear()
    del peers
    # the same model landed in a DeviceInbox slab: the rows kernel
    from p2pdl_amd.node.inbox import DeviceInbox

    template = {f"k{l}": w for l, w in enumerate(w0)}
    inbox = DeviceInbox(template, k_max=K, device=dev)
    for p in range(K):
        ops.fill_synthetic_(inbox.slab[p], 0x5EED0001, p, 1e-2)
    offs = [inbox.layout[f"k{l}"][0] for l in range(len(sizes))]
    ws = [w.clone() for w in w0]
    ops.aggregate_slab_rows_(ws, inbox.slab, list(range(K)), offs, "fedavg")
    # the chunk list over the SAME slab memory (plain views of the rows): the
    # chunk kernel against the rows kernel with the memory layout held fixed,
    # alternated rep by rep
    vptrs = np.array([[inbox.slab[p, offs[l]:offs[l] + sizes[l]].data_ptr() for p in range(K)]
                      for l in range(len(sizes))], dtype=np.uint64)
    ws2 = [w.clone() for w in w0]
    saved_route = ops.STATE_DICT_ROUTE
    ms["rows (inbox slab)"], ms["chunks (slab views)"] = [], []
    try:
        ops.STATE_DICT_ROUTE = "chunks"
        ops.aggregate_ptr_table_(ws2, vptrs, "fedavg")
        for _ in range(reps):
            timed(lambda: ops.aggregate_slab_rows_(ws, inbox.slab, list(range(K)), offs, "fedavg"),
                  ms["rows (inbox slab)"], dev)
            timed(lambda: ops.aggregate_ptr_table_(ws2, vptrs, "fedavg"), ms["chunks (slab views)"], dev)
    finally:
        ops.STATE_DICT_ROUTE = saved_route
        ops._TABLES.clear()
    table = ops.pointer_table([inbox.slab[p, :nflat] for p in range(K)], dev)
    wf = torch.empty(nflat, dtype=torch.float32, device=dev)
    ms["flat (same bytes)"] = []
    for _ in range(reps):
        timed(lambda: ops.aggregate(None, "fedavg", w=wf, lr=0.1, table=table), ms["flat (same bytes)"], dev)
    del inbox, table, wf
    alg = 4.0 * nflat * (K + 2)
    print(f"K={K} x{scale}: {len(sizes)} separately allocated tensors, {nflat:,} coords, "
          f"routes bit-identical: {same}")
    for name, v in ms.items():
        v = sorted(v)
        t = v[len(v) // 2]
        print(f"  {name:18s} median {t:.4f} ms  {alg / t / 1e6:.1f} GB/s  {alg / t / 1e6 / 8000:.4f} of 8 TB/s  "
              f"best {v[0]:.4f}", flush=True)
    for r, t in fresh.items():
        print(f"  {r:18s} fresh table every call: {t:.4f} ms host wall per call", flush=True)
    torch.cuda.empty_cache()
    return same


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 15
    cases = [tuple(int(x) for x in a.split(":")) for a in sys.argv[2:]] or [(64, 1), (16, 1), (64, 4)]
    dev = torch.device("cuda", 0)
    ok = True
    for K, scale in cases:
        ok &= one_case(K, scale, reps, dev)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
