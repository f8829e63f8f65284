"""Probe: how torch-ROCm executes the reference's FedAvg ops
(aggregator/aggregation.py:15-38) on GPU tensors -- is `acc /= K` an IEEE
division or a multiply by fl(1/K)?  Measurement tool, not product."""
import numpy as np
import torch

rng = np.random.default_rng(1)
dev = torch.device("cuda", 0)
for K in (3, 7, 10, 64, 100, 256):
    peers = [rng.standard_normal(1 << 20).astype(np.float32) * np.float32(1e-2) for _ in range(K)]
    w = rng.standard_normal(1 << 20).astype(np.float32) * np.float32(5e-2)
    # the reference's op sequence on CUDA tensors
    acc = torch.zeros_like(torch.from_numpy(w).to(dev))
    for p in peers:
        acc += torch.from_numpy(p).to(dev)
    s = acc.clone()
    acc /= K
    wt = torch.from_numpy(w).to(dev)
    wt += 0.1 * acc
    # numpy restatements
    sn = np.zeros_like(w)
    for p in peers:
        sn = sn + p
    assert np.array_equal(sn, s.cpu().numpy())
    true_div = sn / np.float32(K)
    recip = sn * (np.float32(1.0) / np.float32(K))
    got = acc.cpu().numpy()
    print(f"K={K}: acc/K true-div equal {np.array_equal(got, true_div)}, reciprocal equal {np.array_equal(got, recip)}, "
          f"true vs recip differ in {np.count_nonzero(true_div != recip)} of {w.size}")
    wr = w + np.float32(0.1) * recip
    print(f"   w after apply == recip oracle: {np.array_equal(wt.cpu().numpy(), wr)}")
