#!/usr/bin/env python3
"""Host profile (round 6) of the drop-in's general path with a NEW device
table every call -- a round whose pickle.loads updates arrive at new
addresses: aggregate_models over plain dicts of separately allocated
tensors (ResNet-18 x 64), ops._TABLES cleared before each call, cProfile
over the calls.  Measurement tool, not product.
With "cached" the table is kept (the steady state of a round whose updates
sit at the same addresses: the per-call host cost alone).
With "synced" the profiled calls are synchronised one by one (the host's
own cost per call, no backpressure from queued launches).
usage: python tools/prof_general.py [calls] [mlp] [cached] [synced]"""
import cProfile
import io
import os
import pstats
import sys
import time
import types

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from p2pdl_amd import ops  # noqa: E402
from p2pdl_amd.aggregator import aggregation as agg  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    mlp = "mlp" in sys.argv[2:]  # cfg1: the MNIST MLP x 3
    cached = "cached" in sys.argv[2:]
    dev = torch.device("cuda", 0)
    K = 3 if mlp else 64
    shapes = bench.MLP_SHAPES if mlp else bench.resnet18_param_shapes()
    model = torch.nn.Module()
    for nm, sh in shapes:
        model.register_parameter(nm.replace(".", "__"), torch.nn.Parameter(
            torch.zeros(sh, dtype=torch.float32, device=dev), requires_grad=False))
    keys = [nm.replace(".", "__") for nm, _ in shapes]
    upd = [{k: torch.full(sh, 1e-3 * j, dtype=torch.float32, device=dev) for k, (_, sh) in zip(keys, shapes)}
           for j in range(K)]
    agg.broadcast_global_model_update = lambda self: None
    node = types.SimpleNamespace(model=model, trainers_list=[0] * K, addr="127.0.0.1", port=1, neighbors=[],
                                 received_models=[])

    def call():
        node.received_models.extend({"model": u, "sender": j} for j, u in enumerate(upd))
        if not cached:
            ops._TABLES.clear()
        agg.aggregate_models(node)

    for _ in range(3):
        call()
    torch.cuda.synchronize()
    t = []
    for _ in range(calls):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        call()
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    print(f"{'cached table' if cached else 'new table every call'}: median {np.median(t) * 1e6:.1f} us per call (host wall, synchronised)")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(calls):
        call()
    torch.cuda.synchronize()
    print(f"back to back: {(time.perf_counter() - t0) / calls * 1e6:.1f} us per call (host wall, one sync at the end)")
    synced = "synced" in sys.argv[2:]  # a sync after every call: no queue backpressure in the host's figures
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(calls):
        call()
        if synced:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(60)
    print(s.getvalue())


if __name__ == "__main__":
    main()
