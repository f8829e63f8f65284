#!/usr/bin/env python3
"""A/B timing of robust-rule kernel variants (tools/libp2pdl_lab.so; not the product).

Each variant runs on the same resident synthetic workload as bench.py's
median256 / trimmed256 / cfg4 records; its output is compared bit for bit, on
the device, with the product kernel's output (variant 0) for every
coordinate, and timed with HIP events on the launch stream.

usage: P2P_LIB=tools/libp2pdl_lab.so python tools/lab_robust.py \
          --rule median --peers 256 --coords 100000000 --variants 0,1 [--steps 10]
Prints one JSON line per variant.
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("P2P_LIB", os.path.join(REPO, "tools", "libp2pdl_lab.so"))

import torch  # noqa: E402

from p2pdl_amd import _native as N  # noqa: E402
from p2pdl_amd import ops  # noqa: E402

HBM = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rule", default="median")
    ap.add_argument("--peers", type=int, default=256)
    ap.add_argument("--coords", type=int, default=100_000_000)
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--seed", type=int, default=0x5EED0005)
    ap.add_argument("--data", default="uniform", choices=["uniform", "quantized", "normal"])
    a = ap.parse_args()
    lib = N.load_library()
    lib.p2p_lab_robust.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32,
                                   ctypes.c_int32, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.p2p_lab_robust.restype = ctypes.c_int32
    dev = torch.device("cuda", 0)
    K, n = a.peers, a.coords
    slab = torch.empty((K, n), dtype=torch.float32, device=dev)
    for p in range(K):
        ops.fill_synthetic_(slab[p], a.seed, p, 1e-2)
        if a.data == "quantized":  # many exact ties
            slab[p].mul_(2 ** 9).round_().div_(2 ** 9)
        elif a.data == "normal":
            slab[p].copy_(torch.randn(n, device=dev, generator=torch.Generator(dev).manual_seed(p)) * 1e-2)
    table = ops.pointer_table(list(slab), dev)
    rid = ops.rule_id(a.rule)
    b = ops.trim_count(K) if rid == 2 else 0
    w0 = torch.empty(n, dtype=torch.float32, device=dev)
    ops.fill_synthetic_(w0, a.seed, 0xFFFFF, 5e-2)
    outs = {}
    stream = torch.cuda.current_stream(dev)
    for v in [int(x) for x in a.variants.split(",")]:
        out = torch.empty(n, dtype=torch.float32, device=dev)
        w = w0.clone()

        def launch():
            return lib.p2p_lab_robust(v, table.data_ptr(), K, n, rid, b, 0.1, w.data_ptr(), out.data_ptr(),
                                      stream.cuda_stream)

        rc = launch()
        if rc != 0:
            print(json.dumps({"variant": v, "error": rc}), flush=True)
            continue
        torch.cuda.synchronize()
        ev = []
        for _ in range(a.steps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            launch()
            e1.record(stream)
            ev.append((e0, e1))
        torch.cuda.synchronize()
        ms = sorted(x.elapsed_time(y) for x, y in ev)
        med = ms[len(ms) // 2]
        outs[v] = out
        same = None
        if 0 in outs and v != 0:
            o0 = outs[0].view(torch.int32)
            same = bool(torch.equal(o0, out.view(torch.int32)))
            if not same:
                bad = (o0 != out.view(torch.int32)).nonzero()
                same = f"MISMATCH at {bad.numel()} coords, first {bad[:4].flatten().tolist()}"
        alg = 4 * n * (K + 2)
        print(json.dumps({"variant": v, "rule": a.rule, "peers": K, "coords": n, "data": a.data,
                          "ms_median": round(med, 3), "ms_min": round(ms[0], 3),
                          "frac_hbm": round(alg / (med / 1e3) / 1e9 / HBM, 4),
                          "bit_equal_to_variant0": same}), flush=True)
        del w


if __name__ == "__main__":
    main()
