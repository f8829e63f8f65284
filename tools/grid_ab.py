#!/usr/bin/env python3
"""Lab (round 5): what the FedAvg rate depends on beyond the kernel -- the
launch split and the peer rows' layout (chunks, row spread, chunk-major
planes), row pitch and alignment.  HIP events on one box.  The launch-plan
A/Bs of profiles/r05/grid (grid size, tile groups, XCD-contiguous tiles,
1024-float remainder tiles) ran on lab knobs since removed from
csrc/fedavg.hip.  usage: python tools/grid_ab.py [reps] [mode]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2pdl_amd import ops  # noqa: E402


def chunked(K, n, S, reps, dev):
    """The same [K, n] slab as one launch or S launches over column chunks
    (the same rows, pitch n): launch-level vs memory-layout effects."""
    slab = torch.empty((K, n + 64), dtype=torch.float32, device=dev)
    for p in range(K):
        ops.fill_synthetic_(slab[p], 0x5EED0002, p, 1e-2)
    C = n // S
    whole = ops.pointer_table([slab[p, :n] for p in range(K)], dev)
    parts = [ops.pointer_table([slab[p, s * C:(s + 1) * C] for p in range(K)], dev) for s in range(S)]
    w = torch.empty(n, dtype=torch.float32, device=dev)
    ops.fill_synthetic_(w, 0x5EED0002, 0xFFFFF, 5e-2)
    variants = {"one launch": lambda: ops.aggregate(None, "fedavg", w=w, lr=0.1, table=whole),
                f"{S} chunk launches": lambda: [ops.aggregate(None, "fedavg", w=w[s * C:(s + 1) * C], lr=0.1,
                                                              table=parts[s]) for s in range(S)]}
    ms = {k: [] for k in variants}
    for _ in range(reps):
        for name, fn in variants.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(1_000_000)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ms[name].append(e0.elapsed_time(e1))
    alg = 4.0 * n * (K + 2)
    print(f"K={K} n={n:,} pitch n+64, one launch vs {S} chunks")
    for g, v in ms.items():
        v = sorted(v)
        t = v[len(v) // 2]
        print(f"  {g:>18}  median {t:.4f} ms  {alg / t / 1e6 / 8000:.4f} of 8 TB/s  best {v[0]:.4f}", flush=True)
    del slab
    torch.cuda.empty_cache()


def spread(K, n, pitch, reps, dev, chunk_major_S=0):
    """K rows of n at `pitch` floats (the rows' address spread), or (chunk_major_S)
    n split into S chunks stored chunk-major [S][K][C]: S launches."""
    if chunk_major_S:
        S = chunk_major_S
        C = n // S
        slab = torch.empty((S, K, C + 64), dtype=torch.float32, device=dev)
        tables = [ops.pointer_table([slab[s, p, :C] for p in range(K)], dev) for s in range(S)]
        for s in range(S):
            for p in range(K):
                ops.fill_synthetic_(slab[s, p], 0x5EED0002, p, 1e-2)
        what = f"chunk-major [{S}][{K}][{C:,}]"
    else:
        S, C = 1, n
        slab = torch.empty((K, pitch), dtype=torch.float32, device=dev)
        for p in range(K):
            ops.fill_synthetic_(slab[p, :n + 64], 0x5EED0002, p, 1e-2)
        tables = [ops.pointer_table([slab[p, :n] for p in range(K)], dev)]
        what = f"rows of {n:,} at pitch {pitch:,}"
    w = torch.empty(n, dtype=torch.float32, device=dev)
    ops.fill_synthetic_(w, 0x5EED0002, 0xFFFFF, 5e-2)
    v = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(1_000_000)
        e0.record()
        for s in range(S):
            ops.aggregate(None, "fedavg", w=w[s * C:(s + 1) * C], lr=0.1, table=tables[s])
        e1.record()
        torch.cuda.synchronize()
        v.append(e0.elapsed_time(e1))
    v = sorted(v)
    t = v[len(v) // 2]
    alg = 4.0 * n * (K + 2)
    print(f"K={K} {what}: median {t:.4f} ms  {alg / t / 1e6 / 8000:.4f} of 8 TB/s  best {v[0]:.4f}", flush=True)
    del slab
    torch.cuda.empty_cache()


def plane_sizes(K, n, layouts, reps, dev):
    """The same n coordinates as chunk-major planes of different sizes (each
    layout a list of plane lengths summing to n), carved back to back out of
    ONE buffer so every layout reads the same memory; interleaved per rep.
    Timing only: a layout's planes reinterpret the buffer, so outputs differ
    between layouts (the kernels' bits are pinned by the GPU tests)."""
    assert all(sum(L) == n for L in layouts)
    total = max(sum(K * (c + 64) for c in L) for L in layouts) + 64
    buf = torch.empty(total, dtype=torch.float32, device=dev)
    step = 1 << 30
    for i in range(0, total, step):
        ops.fill_synthetic_(buf[i:i + step], 0x5EED0002, i // step, 1e-2)
    w = torch.empty(n, dtype=torch.float32, device=dev)
    ops.fill_synthetic_(w, 0x5EED0002, 0xFFFFF, 5e-2)
    plans = []
    for L in layouts:
        off, st, tabs = 0, 0, []
        for c in L:
            rows = [buf[off + p * (c + 64):off + p * (c + 64) + c] for p in range(K)]
            assert all(r.numel() == c for r in rows)
            tabs.append((st, c, ops.pointer_table(rows, dev)))
            off += K * (c + 64)
            st += c
        plans.append(tabs)
    ms = [[] for _ in layouts]
    for _ in range(reps):
        for i, tabs in enumerate(plans):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(1_000_000)
            e0.record()
            for st, c, t in tabs:
                ops.aggregate(None, "fedavg", w=w[st:st + c], lr=0.1, table=t)
            e1.record()
            torch.cuda.synchronize()
            ms[i].append(e0.elapsed_time(e1))
    alg = 4.0 * n * (K + 2)
    for L, v in zip(layouts, ms):
        v = sorted(v)
        t = v[len(v) // 2]
        desc = " + ".join(f"{L.count(c)} x {c:,}" for c in dict.fromkeys(L))
        print(f"K={K} n={n:,} planes {desc}: median {t:.4f} ms  {alg / t / 1e6 / 8000:.4f} of 8 TB/s  "
              f"best {v[0]:.4f}", flush=True)
    del buf
    torch.cuda.empty_cache()


def vgpr_views(reps, dev):
    """The VGPR kernel alone (fewer tiles than one split round) at K = 256 over
    row views at several offsets / pitches of one slab."""
    K, n = 256, 1_800_000
    cases = [(3_906_314, 0), (3_906_314, 2_097_152), (3_906_314 + 1024, 2_097_152), (7_812_564, 6_291_456),
             (7_812_564, 0), (2_000_000, 0), (1_800_064, 0)]
    total = max((K - 1) * pitch + off + n for pitch, off in cases) + 64
    slab = torch.empty(total, dtype=torch.float32, device=dev)
    ops.fill_synthetic_(slab, 0x5EED0002, 1, 1e-2)
    w = torch.empty(n, dtype=torch.float32, device=dev)
    ops.fill_synthetic_(w, 0x5EED0002, 0xFFFFF, 5e-2)
    views = [[slab[p * pitch + off:p * pitch + off + n] for p in range(K)] for pitch, off in cases]
    assert all(v.numel() == n for vs in views for v in vs), "every view inside the slab"
    tabs = [ops.pointer_table(vs, dev) for vs in views]
    ms = [[] for _ in cases]
    for _ in range(reps):
        for i, t in enumerate(tabs):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(1_000_000)
            e0.record()
            ops.aggregate(None, "fedavg", w=w, lr=0.1, table=t)
            e1.record()
            torch.cuda.synchronize()
            ms[i].append(e0.elapsed_time(e1))
    alg = 4.0 * n * (K + 2)
    for (pitch, off), v in zip(cases, ms):
        v = sorted(v)
        t = v[len(v) // 2]
        print(f"K=256 n=1.8M pitch {pitch:,} offset {off:,}: median {t:.4f} ms  {alg / t / 1e6 / 8000:.4f} of 8 TB/s",
              flush=True)


def pitch_sweep(dev, K=256, n=1_800_000, start=1_800_064, step=65_536, count=97, reps=3, total=None):
    """The VGPR kernel alone at K peers x n over rows at a sweep of pitches."""
    total = total or (K - 1) * (start + step * (count - 1)) + n + 64
    slab = torch.empty(total, dtype=torch.float32, device=dev)
    print(f"slab {total * 4 / 2**30:.2f} GiB at {slab.data_ptr():#x}", flush=True)
    ops.fill_synthetic_(slab, 0x5EED0002, 1, 1e-2)
    w = torch.empty(n, dtype=torch.float32, device=dev)
    ops.fill_synthetic_(w, 0x5EED0002, 0xFFFFF, 5e-2)
    alg = 4.0 * n * (K + 2)
    for j in range(count):
        pitch = start + step * j
        vs = [slab[p * pitch:p * pitch + n] for p in range(K)]
        assert all(v.numel() == n for v in vs)
        t = ops.pointer_table(vs, dev)
        v = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(500_000)
            e0.record()
            ops.aggregate(None, "fedavg", w=w, lr=0.1, table=t)
            e1.record()
            torch.cuda.synchronize()
            v.append(e0.elapsed_time(e1))
        v = sorted(v)[len(v) // 2]
        print(f"K={K} n={n:,} pitch {pitch:>10,} floats = {pitch * 4:>12,} B = {pitch * 4 / 2**20:9.3f} MiB: "
              f"{alg / v / 1e6 / 8000:.3f}", flush=True)


def layout_ab(K, n, S, reps, dev, rules=("fedavg", "median", "trimmed")):
    """Row-major [K][n] (one launch) against chunk-major planes [S][K][n/S]
    (S launches), both resident, interleaved; the same values in both."""
    C = n // S
    rm = torch.empty((K, n + 64), dtype=torch.float32, device=dev)
    cm = torch.empty((S, K, C + 64), dtype=torch.float32, device=dev)
    for p in range(K):
        ops.fill_synthetic_(rm[p, :n], 0x5EED0002, p, 1e-2)
        for s in range(S):
            cm[s, p, :C].copy_(rm[p, s * C:(s + 1) * C])
    t_rm = ops.pointer_table([rm[p, :n] for p in range(K)], dev)
    t_cm = [ops.pointer_table([cm[s, p, :C] for p in range(K)], dev) for s in range(S)]
    w0 = torch.empty(n, dtype=torch.float32, device=dev)
    ops.fill_synthetic_(w0, 0x5EED0002, 0xFFFFF, 5e-2)
    for rule in rules:
        fns = {"row-major, 1 launch": lambda w: ops.aggregate(None, rule, w=w, lr=0.1, table=t_rm),
               f"planes [{S}][{K}][{C:,}], {S} launches":
                   lambda w: [ops.aggregate(None, rule, w=w[s * C:(s + 1) * C], lr=0.1, table=t_cm[s])
                              for s in range(S)]}
        got = []
        for fn in fns.values():
            x = w0.clone()
            fn(x)
            torch.cuda.synchronize()
            got.append(x.cpu().numpy().view(np.uint32))
        same = np.array_equal(got[0], got[1])
        ms = {k: [] for k in fns}
        w = w0.clone()
        for _ in range(reps):
            for name, fn in fns.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda._sleep(1_000_000)
                e0.record()
                fn(w)
                e1.record()
                torch.cuda.synchronize()
                ms[name].append(e0.elapsed_time(e1))
        alg = 4.0 * n * (K + 2)
        print(f"{rule} K={K} n={n:,}: bit-identical {same}")
        for name, v in ms.items():
            v = sorted(v)
            t = v[len(v) // 2]
            print(f"  {name:36s} median {t:.4f} ms  {alg / t / 1e6 / 8000:.4f} of 8 TB/s  best {v[0]:.4f}", flush=True)
    del rm, cm
    torch.cuda.empty_cache()


def planes_onelaunch(K, n, S, reps, dev, rules=("fedavg", "median", "trimmed")):
    """Chunk-major planes: S launches (one per plane) against ONE segment-table
    launch over all planes (ops.aggregate_segments_), interleaved, bit-compared."""
    from p2pdl_amd import sharded

    C = n // S
    pl = sharded.PeerPlanes(K, S, C, dev)
    for s_ in range(S):
        for p in range(K):
            ops.fill_synthetic_(pl.row(s_, p), 0x5EED0002, p, 1e-2, C, 1, s_)
    w0 = torch.empty((S, C), dtype=torch.float32, device=dev)
    for s_ in range(S):
        ops.fill_synthetic_(w0[s_], 0x5EED0002, 0xFFFFF, 5e-2, C, 1, s_)
    peer_lists = [[pl.row(s_, p) for s_ in range(S)] for p in range(K)]
    for rule in rules:
        fns = {f"{S} launches": lambda w: [pl.reduce_(s_, w[s_], rule) for s_ in range(S)],
               "one segment launch": lambda w: ops.aggregate_segments_([w[s_] for s_ in range(S)], peer_lists, rule)}
        got = []
        for fn in fns.values():
            x = w0.clone()
            fn(x)
            torch.cuda.synchronize()
            got.append(x.cpu().numpy().view(np.uint32))
        same = np.array_equal(got[0], got[1])
        ms = {k: [] for k in fns}
        w = w0.clone()
        for _ in range(reps):
            for name, fn in fns.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda._sleep(1_000_000)
                e0.record()
                fn(w)
                e1.record()
                torch.cuda.synchronize()
                ms[name].append(e0.elapsed_time(e1))
        alg = 4.0 * n * (K + 2)
        print(f"{rule} K={K} n={n:,} planes {S}: bit-identical {same}")
        for name, v in ms.items():
            v = sorted(v)
            t = v[len(v) // 2]
            print(f"  {name:24s} median {t:.4f} ms  {alg / t / 1e6 / 8000:.4f} of 8 TB/s  best {v[0]:.4f}", flush=True)
    del pl
    torch.cuda.empty_cache()


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    mode = sys.argv[2] if len(sys.argv) > 2 else "chunks"
    dev = torch.device("cuda", 0)
    if mode == "chunks":
        chunked(256, 125_000_000, 8, reps, dev)
        chunked(256, 15_625_000 * 2, 2, reps, dev)
    elif mode == "spread":
        for _ in range(2):
            spread(256, 31_250_000, 31_250_064, reps, dev)
            spread(256, 31_250_000, 125_000_064, reps, dev)
            spread(256, 125_000_000, 125_000_064, reps, dev)
            spread(256, 125_000_000, 0, reps, dev, chunk_major_S=8)
    elif mode == "span":
        C = 15_625_000
        for _ in range(2):
            for pitch in (C + 64, 2 * C, 4 * C, 8 * C):
                spread(256, C, pitch, reps, dev)
            spread(256, C // 2, C // 2 + 64, reps, dev)
    elif mode == "planes":
        for _ in range(2):
            for S in (2, 4, 8, 16, 32):
                spread(256, 125_000_000, 0, reps, dev, chunk_major_S=S)
    elif mode == "layout":
        layout_ab(256, 100_000_000, 8, reps, dev)
        layout_ab(128, 100_000_000, 4, reps, dev, rules=("median", "trimmed", "fedavg"))
    elif mode == "rounds":
        for _ in range(3):
            spread(256, 15_625_000, 15_625_064, reps, dev)   # 7 split rounds + 115 tiles + tail
            spread(256, 14_680_064, 14_680_128, reps, dev)   # exactly 7 rounds of 256 x 8192
            spread(256, 16_777_216, 16_777_280, reps, dev)   # exactly 8 rounds
    elif mode == "wholeplanes":
        # the cfg3 tile: 8 equal planes (each 7 split rounds + a 0.45-round
        # VGPR remainder) against planes of whole CU rounds (256 x 8192
        # floats) with one short last plane carrying the only remainder
        n, R = 125_000_000, 256 * 8192
        layouts = [[n // 8] * 8,
                   [8 * R] * 7 + [n - 7 * 8 * R],
                   [7 * R] * 8 + [n - 8 * 7 * R]]
        for _ in range(3):
            plane_sizes(256, n, layouts, reps, dev)
    elif mode == "planerounds":
        # rounds per plane for the cfg3 tile: 4 / 8 (PLANE_BYTES, the product)
        # / 12 / 16 whole CU rounds, one short last plane each
        n, R = 125_000_000, 256 * 8192
        layouts = [[r * R] * (n // (r * R)) + [n % (r * R)] for r in (8, 4, 12, 16)]
        for _ in range(3):
            plane_sizes(256, n, layouts, reps, dev)
    elif mode == "onelaunch":
        planes_onelaunch(128, 100_000_000, 4, reps, dev)
        planes_onelaunch(256, 100_000_000, 8, reps, dev)
    elif mode == "vgpr":
        vgpr_views(reps, dev)
    elif mode == "pitch":
        pitch_sweep(dev)
    elif mode == "misaligned":
        for K, n in ((256, 1_800_000), (64, 11_689_512), (16, 30_000_000), (256, 15_625_000)):
            for extra in (64, 66, 65):  # 256-B, 8-B and 4-B aligned rows
                pitch_sweep(dev, K=K, n=n, start=n + extra, step=1, count=1, total=K * (n + 66) + 64)
            torch.cuda.empty_cache()
    else:
        raise SystemExit(f"unknown mode {mode}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
