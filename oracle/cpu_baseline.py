"""CPU baselines for bench.py (TEST / BENCH INFRASTRUCTURE ONLY).

Only bench.py's cpu_baseline leg imports this module.  Every baseline is the
reference's own CPU op sequence (or, for the build-defined robust rules, the
direct torch restatement of SURVEY.md §8(a) a8), timed on the host cores of
the box bench.py runs on:

    FedAvg   reference aggregator/aggregation.py:15-38, per state_dict key:
             acc = zeros_like(w); for u in peers: acc += u; acc /= K;
             w += 0.1 * acc
    median   torch.median(dim=0) over the stacked peers (lower median)
    trimmed  torch.sort(dim=0), sequential sum of ranks b..K-b-1, / (K-2b)
    delta    reference node/node.py:279,282: cur - prev, then clone
    SHA-256  hashlib.sha256 (OpenSSL, the function behind the reference's
             hashes.SHA256(), utils/crypto.py:56) over the update bytes

Protocol: run with T threads (torch intra-op pool, or a
thread pool for hashlib, which releases the GIL), then with 1 thread, and
report os.cpu_count(), the affinity mask size and T.  T defaults to the
affinity size capped by OMP_NUM_THREADS when the environment sets it: the
GPU box exports OMP_NUM_THREADS=16, its CPU share per GPU, while
os.cpu_count() there counts the whole machine.
"""
from __future__ import annotations

import hashlib
import os
import time
from concurrent.futures import ThreadPoolExecutor

import torch

import oracle


def host_threads() -> dict:
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    env = os.environ.get("OMP_NUM_THREADS")
    t = min(aff, int(env)) if env and env.isdigit() and int(env) > 0 else aff
    return {"cpu_count": os.cpu_count(), "affinity": aff, "threads": t,
            "threads_rule": "min(affinity, OMP_NUM_THREADS)" if env else "affinity"}


def _time(fn, target_s: float):
    fn()  # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        fn()
        reps += 1
        el = time.perf_counter() - t0
        if el >= target_s:
            return reps, el


def measure(fn, bytes_per_call: float, target_s: float, unit_scale: float = 1e9, single_s: float | None = None):
    """Time fn with the host thread count, then with one thread.  Returns a
    dict: value (bytes_per_call / time / unit_scale), value_1thread, threads,
    cpu_count, affinity, reps."""
    info = host_threads()
    prev = torch.get_num_threads()
    try:
        torch.set_num_threads(info["threads"])
        reps, el = _time(fn, target_s)
        torch.set_num_threads(1)
        reps1, el1 = _time(fn, single_s if single_s is not None else max(1.0, target_s / 3))
    finally:
        torch.set_num_threads(prev)
    return dict(info, value=bytes_per_call * reps / el / unit_scale,
                value_1thread=bytes_per_call * reps1 / el1 / unit_scale, reps=reps, seconds=round(el, 2),
                reps_1thread=reps1)


# ---------------------------------------------------------------- op sequences
def reference_ops_fedavg_(w: torch.Tensor, peers, lr: float = 0.1) -> torch.Tensor:
    """reference aggregator/aggregation.py:15-38 for one key."""
    acc = torch.zeros_like(w)
    for p in peers:
        acc += p
    acc /= len(peers)
    w += lr * acc
    return w


def reference_ops_median(peers) -> torch.Tensor:
    return torch.stack(list(peers)).median(dim=0).values


def reference_ops_trimmed(peers, b: int) -> torch.Tensor:
    s = torch.stack(list(peers)).sort(dim=0).values
    acc = torch.zeros_like(s[0])
    for r in range(b, s.shape[0] - b):
        acc += s[r]
    return acc / (s.shape[0] - 2 * b)


def reference_ops_delta(cur: torch.Tensor, prev: torch.Tensor):
    return cur - prev, cur.clone()


# ---------------------------------------------------------------- baselines
def synth_peers(k: int, n: int, seed: int):
    return [torch.from_numpy(oracle.synth(n, seed, p, 1e-2)) for p in range(k)]


def fedavg(k: int, n: int, target_s: float, seed: int = 0x5EED0002) -> dict:
    peers = synth_peers(k, n, seed)
    w = torch.from_numpy(oracle.synth(n, seed, 0xFFFFF, 5e-2))
    return measure(lambda: reference_ops_fedavg_(w, peers), 4.0 * k * n, target_s)


def fedavg_state_dict(k: int, sizes, target_s: float, seed: int = 0x5EED0001) -> dict:
    """The reference's per-key loop over a whole state_dict (cfg2: the 62
    ResNet-18 parameter tensors) with k updates."""
    n = sum(sizes)
    flat = synth_peers(k, n, seed)
    offs = [0]
    for s in sizes:
        offs.append(offs[-1] + s)
    peers = [[f[offs[i]:offs[i + 1]] for i in range(len(sizes))] for f in flat]
    w = torch.from_numpy(oracle.synth(n, seed, 0xFFFFF, 5e-2))
    ws = [w[offs[i]:offs[i + 1]] for i in range(len(sizes))]

    def call():
        for i, wi in enumerate(ws):
            reference_ops_fedavg_(wi, [p[i] for p in peers])

    return measure(call, 4.0 * k * n, target_s)


def median(k: int, n: int, target_s: float, seed: int = 0x5EED0003) -> dict:
    peers = synth_peers(k, n, seed)
    return measure(lambda: reference_ops_median(peers), 4.0 * k * n, target_s)


def trimmed(k: int, n: int, b: int, target_s: float, seed: int = 0x5EED0003) -> dict:
    peers = synth_peers(k, n, seed)
    return measure(lambda: reference_ops_trimmed(peers, b), 4.0 * k * n, target_s)


def delta(n: int, target_s: float, seed: int = 0x5EED0006) -> dict:
    cur = torch.from_numpy(oracle.synth(n, seed, 1, 1e-1))
    prev = torch.from_numpy(oracle.synth(n, seed, 2, 1e-1))
    return measure(lambda: reference_ops_delta(cur, prev), 16.0 * n, target_s)


def sha256(messages, target_s: float) -> dict:
    """hashlib over the messages with a thread pool of the host thread count
    (hashlib releases the GIL on large buffers), then one thread."""
    info = host_threads()
    nbytes = float(sum(map(len, messages)))

    def run(threads, secs):
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(lambda m: hashlib.sha256(m).digest(), messages))
            reps, t0 = 0, time.perf_counter()
            while True:
                list(ex.map(lambda m: hashlib.sha256(m).digest(), messages))
                reps += 1
                el = time.perf_counter() - t0
                if el >= secs:
                    return reps, el

    reps, el = run(info["threads"], target_s)
    reps1, el1 = run(1, max(1.0, target_s / 3))
    return dict(info, value=nbytes * reps / el / 1e9, value_1thread=nbytes * reps1 / el1 / 1e9, reps=reps,
                seconds=round(el, 2), reps_1thread=reps1)


def arrival(messages, expected, w: "torch.Tensor", target_s: float) -> dict:
    """cfg5 as the reference's node receives it, on the host: SHA-256 of every
    serialized update (hashlib, utils/crypto.py:56 -- with a thread pool of
    the host thread count, then one thread), the updates whose digest matches
    what the sender signed unpickled (node/node.py:138 pickle.loads: CPU
    tensors) and the reference's FedAvg op sequence over them
    (aggregator/aggregation.py:15-38, torch intra-op threads = the host
    thread count, then one).  value = hashed bytes per second (GB/s)."""
    import pickle

    info = host_threads()
    nbytes = float(sum(map(len, messages)))
    w0 = w.clone()

    def one(ex):
        ds = list(ex.map(lambda m: hashlib.sha256(m).digest(), messages)) if ex else \
            [hashlib.sha256(m).digest() for m in messages]
        acc = [pickle.loads(m)["w"] for m, d, e in zip(messages, ds, expected) if d == e]
        w.copy_(w0)
        reference_ops_fedavg_(w, acc)
        return len(acc)

    def run(threads, secs):
        prev = torch.get_num_threads()
        torch.set_num_threads(threads)
        try:
            with ThreadPoolExecutor(threads) as ex:
                pool = ex if threads > 1 else None
                one(pool)
                reps, t0 = 0, time.perf_counter()
                while True:
                    n_acc = one(pool)
                    reps += 1
                    el = time.perf_counter() - t0
                    if el >= secs:
                        return reps, el, n_acc
        finally:
            torch.set_num_threads(prev)

    reps, el, n_acc = run(info["threads"], target_s)
    reps1, el1, _ = run(1, max(1.0, target_s / 3))
    return dict(info, value=nbytes * reps / el / 1e9, value_1thread=nbytes * reps1 / el1 / 1e9, reps=reps,
                seconds=round(el, 2), reps_1thread=reps1, accepted=n_acc)
