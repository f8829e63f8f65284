"""HBM rate of the float16 / bfloat16 FedAvg kernel (p2p_fedavg_apply_16)
over K peers x n coordinates resident on the GPU: algorithmic bytes
2n(K+2) per launch / HIP-event time.  Measurement tool, not product."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2pdl_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
for dt in (torch.float16, torch.bfloat16):
    for K, n in ((64, 125_000_000), (256, 62_500_000)):
        peers = [torch.randn(n, device=dev).to(dt) * 0.01 for _ in range(K)]
        w = torch.randn(n, device=dev).to(dt)
        for _ in range(2):
            ops.fedavg16_apply_(w, peers)
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in ev:
            a.record()
            ops.fedavg16_apply_(w, peers)
            b.record()
        torch.cuda.synchronize()
        ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
        gbs = 2 * n * (K + 2) / ms / 1e6
        print(f"{str(dt):15s} K={K:3d} n={n:,}: {ms:8.3f} ms  {gbs:7.1f} GB/s  {gbs / 8000:.3f} of 8 TB/s", flush=True)
        del peers, w
        torch.cuda.empty_cache()
