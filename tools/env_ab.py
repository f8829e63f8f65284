#!/usr/bin/env python3
"""Same-process A/B of node/envelope.envelope_parts against another version
of the module (a file path), on a ResNet-18-sized GPU state_dict: ms per call
to the parts the broadcast sends, alternating, best of R rounds each.

usage: env_ab.py <other envelope.py> [rounds]"""
import importlib.util
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402  (resnet18_param_shapes)
from p2pdl_amd import ops  # noqa: E402
from p2pdl_amd.node import envelope as prod  # noqa: E402


def main():
    spec = importlib.util.spec_from_file_location("envelope_other", sys.argv[1])
    other = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(other)
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda", 0)
    sd = {}
    for i, (nm, shape) in enumerate(bench.resnet18_param_shapes()):
        t = torch.empty(shape, dtype=torch.float32, device=dev)
        ops.fill_synthetic_(t.view(-1), 0x5EED, i, 5e-2)
        sd[nm] = t
    torch.cuda.synchronize()
    nbytes = sum(t.numel() * 4 for t in sd.values())

    def timed(mod, steps=20):
        with mod.LOCK:
            for _ in range(3):
                mod.envelope_parts(sd, "h", 1)
            t0 = time.perf_counter()
            for _ in range(steps):
                mod.envelope_parts(sd, "h", 1)
            return (time.perf_counter() - t0) / steps * 1e3

    with prod.LOCK, other.LOCK:
        a = b"".join(prod.envelope_parts(sd, "h", 1))
        b = b"".join(other.envelope_parts(sd, "h", 1))
    print(f"identical envelopes: {a == b}")
    res = {"prod": [], "other": []}
    for _ in range(rounds):
        res["other"].append(timed(other))
        res["prod"].append(timed(prod))
    for k, v in res.items():
        print(f"{k:6s} ms/call " + " ".join(f"{x:.3f}" for x in v) + f"   best {min(v):.3f} = {nbytes / min(v) / 1e6:.1f} GB/s")


if __name__ == "__main__":
    main()
