"""CPU baseline: the reference's aggregation op sequence on torch CPU.

TEST / BENCH INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).  This is the
exact ATen op sequence of reference aggregator/aggregation.py:15-38 applied to
one flat fp32 buffer (what the reference runs per state_dict key):

    acc = torch.zeros_like(w)        # :15
    for upd in peers: acc += upd     # :25-28
    acc /= K                         # :31-32
    w += 0.1 * acc                   # :36-38

run with torch's intra-op thread pool (the reference's own CPU path).
"""
from __future__ import annotations

import time

import torch

import oracle


def reference_ops_fedavg_(w: torch.Tensor, peers, lr: float = 0.1) -> torch.Tensor:
    acc = torch.zeros_like(w)
    for p in peers:
        acc += p
    acc /= len(peers)
    w += lr * acc
    return w


def reference_ops_median(peers) -> torch.Tensor:
    """Build-defined rule on CPU (torch.median lower median; NaN-free data)."""
    return torch.stack(list(peers)).median(dim=0).values


def time_fedavg(k: int, n: int, target_s: float = 12.0, seed: int = 0x5EED0002):
    """Time reference_ops_fedavg_ over a resident (k, n) sample for ~target_s.

    Returns (GB/s of peer-update bytes, threads, reps, seconds)."""
    peers = [torch.from_numpy(oracle.synth(n, seed, p, 1e-2)) for p in range(k)]
    w = torch.from_numpy(oracle.synth(n, seed, 0xFFFFF, 5e-2))
    reference_ops_fedavg_(w, peers)  # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        reference_ops_fedavg_(w, peers)
        reps += 1
        el = time.perf_counter() - t0
        if el >= target_s:
            break
    return k * n * 4 * reps / el / 1e9, torch.get_num_threads(), reps, el


def time_median(k: int, n: int, target_s: float = 12.0, seed: int = 0x5EED0003):
    peers = [torch.from_numpy(oracle.synth(n, seed, p, 1e-2)) for p in range(k)]
    reps, t0 = 0, time.perf_counter()
    while True:
        reference_ops_median(peers)
        reps += 1
        el = time.perf_counter() - t0
        if el >= target_s:
            break
    return k * n * 4 * reps / el / 1e9, torch.get_num_threads(), reps, el


def reference_ops_delta(cur: torch.Tensor, prev: torch.Tensor):
    """Reference node/node.py:279,282 on one flat buffer: sub, then clone."""
    return cur - prev, cur.clone()


def time_delta(n: int, target_s: float = 12.0, seed: int = 0x5EED0006):
    """GB/s of algorithmic traffic (16 B per coordinate: read cur, read prev,
    write delta, write the new snapshot) of the reference's torch CPU ops."""
    cur = torch.from_numpy(oracle.synth(n, seed, 1, 1e-1))
    prev = torch.from_numpy(oracle.synth(n, seed, 2, 1e-1))
    reference_ops_delta(cur, prev)
    reps, t0 = 0, time.perf_counter()
    while True:
        reference_ops_delta(cur, prev)
        reps += 1
        el = time.perf_counter() - t0
        if el >= target_s:
            break
    return 16 * n * reps / el / 1e9, torch.get_num_threads(), reps, el
