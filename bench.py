#!/usr/bin/env python3
"""Benchmark of the aggregation hot path (driver contract: one JSON line).

Metric (BASELINE.json): aggregated peer-update GB/s (% HBM peak) at 1/2/4/8
MI355X.  Default workload = cfg3's per-GPU coordinate tile: 256 peers x 125M
fp32 coordinates PER GPU (weak scaling; at 8 GPUs the job is exactly cfg3,
1B coordinates x 256 peers).  cfg3 itself (1.02 TB of peer data) does not fit
one GPU's 288 GB, so a GPU owns one 125M-coordinate tile (128 GB resident).

A step = one FedAvg pass (sum of K peers in list order, /K, w += 0.1*mean)
over the resident tile; at N > 1 each rank reduces its round-robin coordinate
chunks and an RCCL all-gather (over xGMI) reassembles the global model,
pipelined per chunk on a second stream.  Inputs are generated on device by
the counter PRNG before timing; nothing is skipped inside the timed region.

value = peer-update bytes consumed by all ranks / step time (GB/s).
roofline.achieved = algorithmic bytes per launch 4n(K+2) / mean kernel time
(HIP events on the launch stream), peak 8.0 TB/s.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from p2pdl_amd import ops  # noqa: E402

HBM_PEAK_GBS = 8000.0
W_PEER, UPD_SCALE, W_SCALE = 0xFFFFF, 1e-2, 5e-2

WORKLOADS = {
    # name: (rule, peers, coords per GPU, seed)
    "cfg3": ("fedavg", 256, 125_000_000, 0x5EED0002),
    "cfg2": ("fedavg", 64, 11_689_512, 0x5EED0001),
    "cfg4-median": ("median", 128, 100_000_000, 0x5EED0003),
    "cfg4-trimmed": ("trimmed", 128, 100_000_000, 0x5EED0003),
    # north-star robust target: median over 256 peers (cfg3's K) on a 100M tile
    "median256": ("median", 256, 100_000_000, 0x5EED0005),
    "trimmed256": ("trimmed", 256, 100_000_000, 0x5EED0005),
    # cfg5: 256 serialized updates (64-B header + 25M fp32 payload), digest all,
    # reject the ~10% whose bytes were corrupted, FedAvg the accepted ones
    "cfg5": ("fused", 256, 25_000_000, 0x5EED0004),
    # SHA-256 alone over 256 messages of the cfg5 size
    "sha256": ("sha256", 256, 25_000_000, 0x5EED0004),
    # trainer-side delta + snapshot of cfg3's 1B-param model
    "delta": ("delta", 1, 1_000_000_000, 0x5EED0006),
    # cfg1: the reference's default run -- MNIST MLP (models/model.py:6-8), 3
    # peers, the drop-in aggregate_models end to end (latency-bound)
    "cfg1": ("dropin", 3, 535_818, 0x5EED0000),
    # land 16 serialized ResNet-18-sized updates (11.7M
    # params each) in the device slab vs the reference's pickle.loads
    "inbox": ("inbox", 16, 11_689_512, 0x5EED0007),
}
MSG_HEADER = 64  # bytes before the payload (keeps payloads 16-B aligned)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="cfg3", choices=sorted(WORKLOADS))
    ap.add_argument("--coords", type=int, default=0, help="override coordinates per GPU")
    ap.add_argument("--peers", type=int, default=0, help="override K")
    ap.add_argument("--chunks", type=int, default=8, help="all-gather pipeline chunks per rank (N>1)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true")
    return ap.parse_args()


def run_digest_workload(args, rule, K, n, seed, dev):
    """cfg5 / sha256: one process, one GPU (replicas only: see DESIGN.md)."""
    import hashlib

    import numpy as np

    msg_bytes = MSG_HEADER + 4 * n
    stride = -(-msg_bytes // 256) * 256
    buf = torch.zeros(K * stride, dtype=torch.uint8, device=dev)
    log(f"generating {K} messages x {msg_bytes:,} B ({K*stride/1e9:.1f} GB)")
    for p in range(K):
        hdr = np.frombuffer((f"p2pdl-update peer={p:05d} n={n} ".encode() + bytes(64))[:MSG_HEADER], dtype=np.uint8)
        buf[p * stride:p * stride + MSG_HEADER].copy_(torch.from_numpy(hdr.copy()))
        payload = buf[p * stride + MSG_HEADER:p * stride + msg_bytes].view(torch.float32)
        ops.fill_synthetic_(payload, seed, p, UPD_SCALE)
    offsets = [p * stride for p in range(K)]
    lens = [msg_bytes] * K
    ptrs = torch.tensor([buf.data_ptr() + o for o in offsets], dtype=torch.int64, device=dev)
    lens_d = torch.tensor(lens, dtype=torch.int64, device=dev)
    digests = torch.empty((K, 32), dtype=torch.uint8, device=dev)
    lib = ops.N.lib()

    def digest():
        ops.N.check(lib.p2p_sha256_batch(ptrs.data_ptr(), lens_d.data_ptr(), K, digests.data_ptr(),
                                         ops.N.stream_handle()), "sha256")

    digest()
    expected = digests.clone()  # what the senders signed (untimed)
    torch.cuda.synchronize()
    # cross-check two digests on the host (checker only)
    for p in (0, K - 1):
        assert bytes(digests[p].cpu().numpy()) == hashlib.sha256(
            bytes(buf[offsets[p]:offsets[p] + msg_bytes].cpu().numpy())).digest(), "sha256 mismatch"
    log("digest spot check vs hashlib: ok")
    bad = [p for p in range(K) if (p * 7919) % 10 == 3]  # ~10% corrupted in flight
    for p in bad:
        buf[offsets[p] + MSG_HEADER + 1000] ^= 0x40
    payload_tbl = torch.tensor([buf.data_ptr() + o + MSG_HEADER for o in offsets], dtype=torch.int64, device=dev)
    accepted = torch.zeros(K, dtype=torch.int64, device=dev)
    count = torch.zeros(1, dtype=torch.int32, device=dev)
    w = torch.empty(n, dtype=torch.float32, device=dev)
    ops.fill_synthetic_(w, seed, W_PEER, W_SCALE)
    comp = torch.cuda.current_stream(dev)
    kern = []

    def step(record=False):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)] if record else None
        if record:
            e[0].record(comp)
        digest()
        if record:
            e[1].record(comp)
        if rule == "fused":
            ops.digest_accept(digests, expected, payload_tbl, accepted, count)
            ops.fedavg_apply_devk_(w, accepted, count, K)
        if record:
            e[2].record(comp)
            kern.append(e)

    for _ in range(max(args.warmup, 1)):
        step()
    torch.cuda.synchronize()
    if rule == "fused":
        assert int(count.item()) == K - len(bad), "accept count"
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(record=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    step_s = el / args.steps
    sha_ms = sum(a.elapsed_time(b) for a, b, _ in kern) / len(kern)
    agg_ms = sum(b.elapsed_time(c) for _, b, c in kern) / len(kern)
    hashed = K * msg_bytes
    acc = K - len(bad)
    agg_bytes = 4 * n * (acc + 2) if rule == "fused" else 0
    cpu = None
    if not args.no_cpu_baseline:
        from concurrent.futures import ThreadPoolExecutor

        thr = int(os.environ.get("OMP_NUM_THREADS", "16"))
        sample = [bytes(buf[offsets[p]:offsets[p] + min(msg_bytes, 16 << 20)].cpu().numpy()) for p in range(min(K, 32))]
        t0 = time.perf_counter()
        reps = 0
        with ThreadPoolExecutor(thr) as ex:  # hashlib releases the GIL
            while time.perf_counter() - t0 < args.cpu_seconds:
                list(ex.map(lambda m: hashlib.sha256(m).digest(), sample))
                reps += 1
        ce = time.perf_counter() - t0
        cpu = {"value": round(sum(map(len, sample)) * reps / ce / 1e9, 3), "unit": "GB/s", "cores": thr,
               "kind": "port", "sample": f"hashlib.sha256 (OpenSSL, the function behind reference "
                                         f"utils/crypto.py:56) over {len(sample)} x {len(sample[0]):,} B, "
                                         f"{thr} threads, {reps} reps"}
    line = {
        "metric": "aggregated peer-update GB/s (% HBM peak) at 1/2/4/8 MI355X",
        "value": round(hashed / step_s / 1e9, 3), "unit": "GB/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32 (SHA-256) + fp32",
        "data": "synthetic serialized updates (64-B header + device-PRNG fp32 payload)",
        "config": {"workload": f"{args.workload}: {K} messages x {msg_bytes:,} B"
                               + (f", {len(bad)} corrupted, FedAvg over {acc} accepted" if rule == "fused" else ""),
                   "peers": K, "coords_per_peer": n, "parallelism": "single GPU (replicas only)"},
        "roofline": {"bound": "int-alu (serial SHA-256 chain per message; see DESIGN.md)",
                     "achieved": round(hashed / (sha_ms / 1e3) / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(hashed / (sha_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 5), "traffic": None,
                     "kernel_ms": round(sha_ms, 3), "fedavg_ms": round(agg_ms, 3),
                     "fedavg_gbs": round(agg_bytes / (agg_ms / 1e3) / 1e9, 1) if agg_bytes else None,
                     # serial-chain issue bound: one wave issues ~1 instruction / 4 cycles at
                     # 2.4 GHz, ~910 instructions per 64-B block on the chain
                     "chain_issue_bound_gbs": round(min(K, 65536) * 64 / (910 * 4 / 2.4e9) / 1e9, 2)},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)


def run_delta_workload(args, n, seed, dev):
    """Trainer-side local update (reference node/node.py:273-282) of one
    flat n-parameter model: delta = cur - prev; prev = cur.  One GPU."""
    import numpy as np

    cur = torch.empty(n, dtype=torch.float32, device=dev)
    prev = torch.empty_like(cur)
    delta = torch.empty_like(cur)
    ops.fill_synthetic_(cur, seed, 1, 1e-1)
    ops.fill_synthetic_(prev, seed, 2, 1e-1)
    comp = torch.cuda.current_stream(dev)
    if not args.no_check:  # one launch, checked against the oracle on a prefix
        import oracle  # checker only

        m = min(n, 1 << 20)
        ops.delta_snapshot_(cur, prev, delta)
        torch.cuda.synchronize()
        want, _ = oracle.delta_snapshot_np(oracle.synth(m, seed, 1, 1e-1), oracle.synth(m, seed, 2, 1e-1))
        ok = np.array_equal(delta[:m].cpu().numpy().view(np.uint32), want.view(np.uint32)) and \
            torch.equal(prev[:m], cur[:m])
        log(f"spot check vs oracle ({m} coords): {'bit-exact' if ok else 'MISMATCH'}")
        if not ok:
            raise SystemExit("bench: delta kernel differs from the oracle")
    for _ in range(max(args.warmup, 1)):
        ops.delta_snapshot_(cur, prev, delta)
    torch.cuda.synchronize()
    ev = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(comp)
        ops.delta_snapshot_(cur, prev, delta)
        e1.record(comp)
        ev.append((e0, e1))
    torch.cuda.synchronize()
    step_s = (time.perf_counter() - t0) / args.steps
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
    alg = 16 * n
    traffic = None
    tfile = os.path.join(REPO, "profiles", "traffic_delta.json")
    if os.path.exists(tfile):
        with open(tfile) as f:
            tj = json.load(f)
        if tj.get("coords_per_launch") == n:
            traffic = tj.get("hbm_bytes_per_launch")
    cpu = None
    if not args.no_cpu_baseline:
        import oracle.cpu_baseline as cb  # baseline leg only

        torch.set_num_threads(min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16"))))
        n_s = 50_000_000
        gbs, thr, reps, el = cb.time_delta(n_s, args.cpu_seconds)
        cpu = {"value": round(gbs, 3), "unit": "GB/s", "cores": thr, "kind": "port",
               "sample": f"{n_s:,} fp32 params, reference ops cur - prev and clone (node/node.py:279,282) "
                         f"on torch CPU, {reps} reps in {el:.1f}s"}
    print(json.dumps({
        "metric": "aggregated peer-update GB/s (% HBM peak) at 1/2/4/8 MI355X",
        "value": round(alg / step_s / 1e9, 2), "unit": "GB/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (device counter PRNG); value = algorithmic bytes (16 B/param) per second",
        "config": {"workload": f"delta: trainer local update over {n:,} fp32 params (SURVEY §8(f) row 2)",
                   "coords_per_gpu": n, "parallelism": "single GPU (replicas only)"},
        "roofline": {"bound": "hbm", "achieved": round(alg / (kern_ms / 1e3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(alg / (kern_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "kernel_ms": round(kern_ms, 4), "alg_bytes_per_launch": alg},
        "cpu_baseline": cpu}), flush=True)


MLP_SHAPES = [("fc1.weight", (512, 784)), ("fc1.bias", (512,)), ("fc2.weight", (256, 512)),
              ("fc2.bias", (256,)), ("fc3.weight", (10, 256)), ("fc3.bias", (10,))]  # models/model.py:6-8


def run_dropin_workload(args, K, seed, dev):
    """cfg1: one call of the drop-in aggregate_models (reference
    aggregator/aggregation.py:7-46) on the MNIST MLP with K updates, host
    table building included -- latency, reported as us per call."""
    import types

    from p2pdl_amd.aggregator import aggregation as agg

    agg_bc = agg.broadcast_global_model_update
    agg.broadcast_global_model_update = lambda self: None  # networking is out of scope
    model = torch.nn.Module()
    n = 0
    for name, shape in MLP_SHAPES:
        mod, attr = name.split(".")
        if not hasattr(model, mod):
            model.add_module(mod, torch.nn.Module())
        t = torch.empty(shape, dtype=torch.float32, device=dev)
        ops.fill_synthetic_(t.view(-1), seed, W_PEER, W_SCALE)
        getattr(model, mod).register_parameter(attr, torch.nn.Parameter(t, requires_grad=False))
        n += t.numel()
    updates = []
    for p in range(K):
        upd = {}
        for name, shape in MLP_SHAPES:
            t = torch.empty(shape, dtype=torch.float32, device=dev)
            ops.fill_synthetic_(t.view(-1), seed, p, UPD_SCALE)
            upd[name] = t
        updates.append(upd)
    node = types.SimpleNamespace(model=model, trainers_list=[0] * K, addr="127.0.0.1", port=1, neighbors=[],
                                 received_models=[])

    def call():
        node.received_models.extend({"model": u, "sender": j} for j, u in enumerate(updates))
        agg.aggregate_models(node)

    for _ in range(max(args.warmup, 3)):
        call()
    torch.cuda.synchronize()
    steps = max(args.steps, 100)
    t0 = time.perf_counter()
    for _ in range(steps):
        call()
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / steps * 1e6
    agg.broadcast_global_model_update = agg_bc
    cpu = None
    if not args.no_cpu_baseline:
        import oracle.cpu_baseline as cb  # baseline leg only

        torch.set_num_threads(min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16"))))
        ws = [torch.zeros(s) for _, s in MLP_SHAPES]
        peers = [[torch.rand(s) for _, s in MLP_SHAPES] for _ in range(K)]
        reps, t1 = 0, time.perf_counter()
        while time.perf_counter() - t1 < min(args.cpu_seconds, 3.0):
            for l, w in enumerate(ws):  # the reference's per-key op sequence (aggregation.py:15-38)
                cb.reference_ops_fedavg_(w, [p[l] for p in peers])
            reps += 1
        cus = (time.perf_counter() - t1) / reps * 1e6
        cpu = {"value": round(cus, 1), "unit": "us per aggregation", "cores": torch.get_num_threads(),
               "kind": "port", "sample": f"MLP state_dict ({n:,} params) x {K} updates, reference op sequence "
                                         f"per key on torch CPU, {reps} reps"}
    print(json.dumps({
        "metric": "aggregated peer-update GB/s (% HBM peak) at 1/2/4/8 MI355X",
        "value": round(K * n * 4 / (us * 1e-6) / 1e9, 3), "unit": "GB/s", "n_gpus": 1, "steps": steps,
        "warmup": args.warmup, "ms_per_step": round(us / 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32", "data": "synthetic MLP weights and updates (device PRNG)",
        "config": {"workload": f"cfg1: drop-in aggregate_models, MNIST MLP ({n:,} params) x {K} updates, "
                               f"latency-bound (us_per_call)", "us_per_call": round(us, 1),
                   "parallelism": "single GPU"},
        "roofline": None, "cpu_baseline": cpu}), flush=True)


def _resnet18_like_shapes(total):
    """Tensor sizes of a ResNet-18 state_dict (conv/fc weights, BN vectors),
    the last one padded so the parameters add up to `total`."""
    sizes = [64 * 3 * 49] + [64] * 2 + [64 * 64 * 9] * 4 + [64] * 8 + [128 * 64 * 9, 128 * 128 * 9, 128 * 64]
    sizes += [128 * 128 * 9] * 2 + [128] * 10 + [256 * 128 * 9, 256 * 256 * 9, 256 * 128] + [256 * 256 * 9] * 2
    sizes += [256] * 10 + [512 * 256 * 9, 512 * 512 * 9, 512 * 256] + [512 * 512 * 9] * 2 + [512] * 10
    sizes += [1000 * 512, 1000]
    sizes[-2] += total - sum(sizes)
    return sizes


def run_inbox_workload(args, K, n, seed, dev):
    """Receive path (reference node/node.py:135-138): K serialized updates of
    a GPU sender (pickle of CUDA tensors, node/node.py:285) deserialized into
    device tensors -- the reference's pickle.loads vs DeviceInbox.land.
    value = update bytes landed per second (host-to-device, PCIe-bound)."""
    import pickle

    from p2pdl_amd.node.inbox import DeviceInbox

    sizes = _resnet18_like_shapes(n)
    keys = [f"layer{i}.weight" for i in range(len(sizes))]
    ser = []
    for p in range(K):
        upd = {}
        for i, (k, m) in enumerate(zip(keys, sizes)):
            t = torch.empty(m, dtype=torch.float32, device=dev)
            ops.fill_synthetic_(t, seed, p * 1000 + i, UPD_SCALE)
            upd[k] = t
        ser.append(pickle.dumps(upd))  # what a CUDA trainer sends
    template = {k: torch.empty(m, dtype=torch.float32, device=dev) for k, m in zip(keys, sizes)}
    inbox = DeviceInbox(template, k_max=K, device=dev)
    if not args.no_check:
        got = inbox.land(ser[0], 0)
        ref = pickle.loads(ser[0])
        torch.cuda.synchronize()
        ok = all(torch.equal(got[k], ref[k]) for k in keys)
        log(f"landed update == pickle.loads: {ok}")
        if not ok:
            raise SystemExit("bench: inbox differs from pickle.loads")

    def timed(fn):
        for _ in range(max(args.warmup, 1)):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.steps

    def ours():
        inbox.reset()
        for s in ser:
            inbox.land(s)

    def reference():
        for s in ser:
            pickle.loads(s)

    t_ours, t_ref = timed(ours), timed(reference)
    nbytes = K * n * 4
    print(json.dumps({
        "metric": "aggregated peer-update GB/s (% HBM peak) at 1/2/4/8 MI355X",
        "value": round(nbytes / t_ours / 1e9, 3), "unit": "GB/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(t_ours * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32", "data": "synthetic ResNet-18-sized updates pickled from CUDA tensors",
        "config": {"workload": f"inbox: land {K} serialized updates of {n:,} params ({len(sizes)} tensors) "
                               f"in the device slab (SURVEY §8(f) row 1)", "reference_pickle_loads_gbs":
                   round(nbytes / t_ref / 1e9, 3), "reference_ms": round(t_ref * 1e3, 3),
                   "parallelism": "single GPU, host-to-device"},
        "roofline": {"bound": "pcie (host-to-device)", "achieved": round(nbytes / t_ours / 1e9, 2), "peak": 63.0,
                     "unit": "GB/s", "frac": round(nbytes / t_ours / 1e9 / 63.0, 4), "traffic": None},
        "cpu_baseline": None}), flush=True)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # P2P_DIST_BACKEND=gloo rehearses N>1 on a single GPU (ranks share cuda:0);
    # the driver's multi-GPU runs use nccl (= RCCL over xGMI), one GPU per rank.
    backend = os.environ.get("P2P_DIST_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    rule, K, n, seed = WORKLOADS[args.workload]
    K = args.peers or K
    n = args.coords or n
    if rule in ("fused", "sha256"):
        if world > 1:
            raise SystemExit("cfg5/sha256 run as replicas only (one process per GPU)")
        return run_digest_workload(args, rule, K, n, seed, dev)
    if rule == "delta":
        if world > 1:
            raise SystemExit("delta runs as replicas only (one process per GPU)")
        return run_delta_workload(args, n, seed, dev)
    if rule == "inbox":
        if world > 1:
            raise SystemExit("inbox runs on one GPU")
        return run_inbox_workload(args, K, n, seed, dev)
    if rule == "dropin":
        if world > 1:
            raise SystemExit("cfg1 runs on one GPU")
        return run_dropin_workload(args, K, seed, dev)
    S = args.chunks if world > 1 else 1
    C = -(-n // S)
    n = C * S  # whole chunks per rank
    free, total = torch.cuda.mem_get_info(dev)
    need = (K + 2 + world) * n * 4
    if need > free * 0.97:
        raise SystemExit(f"workload needs {need/1e9:.1f} GB, {free/1e9:.1f} GB free")

    # ---- synthetic inputs, resident in HBM (outside the timed region) ----
    log(f"[rank {rank}] generating {K} x {n:,} fp32 peer slab ({K*n*4/1e9:.1f} GB)")
    slab = torch.empty((K, n), dtype=torch.float32, device=dev)
    for p in range(K):
        ops.fill_synthetic_(slab[p], seed, p, UPD_SCALE, C, world, rank)
    w = torch.empty(n, dtype=torch.float32, device=dev)
    ops.fill_synthetic_(w, seed, W_PEER, W_SCALE, C, world, rank)
    w_full = torch.empty(n * world, dtype=torch.float32, device=dev) if world > 1 else None
    tables = [ops.pointer_table([slab[p, s * C:(s + 1) * C] for p in range(K)], dev) for s in range(S)]
    torch.cuda.synchronize()

    comp = torch.cuda.current_stream(dev)
    comm = torch.cuda.Stream(dev)
    kern_events = []  # (start, end) per kernel launch, on the launch stream

    def step(record=False):
        for s in range(S):
            ws = w[s * C:(s + 1) * C]
            if record:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(comp)
            ops.aggregate(None, rule, w=ws, lr=0.1, table=tables[s])
            if record:
                e1.record(comp)
                kern_events.append((e0, e1))
            if world > 1:
                done = torch.cuda.Event()
                done.record(comp)
                comm.wait_event(done)
                with torch.cuda.stream(comm):
                    dist.all_gather_into_tensor(w_full[s * C * world:(s + 1) * C * world], ws)
        if world > 1:
            comp.wait_stream(comm)

    # ---- correctness spot check of the first warmup step vs the oracle ----
    # rank 0 checks the first m coordinates of EVERY rank's first chunk: in its
    # own w and, at N > 1, where the all-gather placed them in the global model
    m = min(4096, C)
    check = not args.no_check and rank == 0
    for i in range(max(args.warmup, 1 if check else 0)):
        step()
        if i == 0 and check:
            torch.cuda.synchronize()
            import numpy as np

            import oracle  # checker only
            rid = ops.rule_id(rule)
            bad = []
            for g in range(world):
                peers = [oracle.synth(m, seed, p, UPD_SCALE, C, world, g) for p in range(K)]
                w0 = oracle.synth(m, seed, W_PEER, W_SCALE, C, world, g)
                if rid == 0:
                    want, _ = oracle.fedavg(peers, w0)
                else:
                    want, _ = oracle.robust(peers, rid, ops.trim_count(K) if rid == 2 else 0, w=w0)
                got = (w_full[g * C:g * C + m] if world > 1 else w[:m]).cpu().numpy()
                if not np.array_equal(got.view(np.uint32), want.view(np.uint32)):
                    bad.append(g)
            log(f"[rank 0] spot check vs oracle ({m} coords x {world} rank chunk(s)): "
                f"{'bit-exact' if not bad else f'MISMATCH on ranks {bad}'}")
            if bad:
                raise SystemExit("bench: kernel output differs from the oracle")
        if world > 1:
            dist.barrier()

    # ---- timed region ----
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(record=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_ms = sum(a.elapsed_time(b) for a, b in kern_events) / len(kern_events)

    step_s = elapsed / args.steps
    peer_bytes = K * n * 4 * world
    value = peer_bytes / step_s / 1e9
    launch_n = C
    alg_bytes = 4 * launch_n * (K + 2)
    achieved = alg_bytes / (kern_ms / 1e3) / 1e9

    traffic = None
    tfile = os.path.join(REPO, "profiles", f"traffic_{args.workload}.json")
    if os.path.exists(tfile):
        with open(tfile) as f:
            tj = json.load(f)
        if tj.get("coords_per_launch") == launch_n and tj.get("peers") == K:
            traffic = tj.get("hbm_bytes_per_launch")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle.cpu_baseline as cb  # baseline leg only

        torch.set_num_threads(min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16"))))
        n_s = 1_000_000
        if rule == "fedavg":
            gbs, thr, reps, el = cb.time_fedavg(K, n_s, args.cpu_seconds)
        else:
            gbs, thr, reps, el = cb.time_median(K, n_s, args.cpu_seconds)
        what = ("reference op sequence (aggregation.py:15-38)" if rule == "fedavg"
                else "torch.median(dim=0) (the build-defined rule on CPU)")
        cpu = {"value": round(gbs, 3), "unit": "GB/s", "cores": thr, "kind": "port",
               "sample": f"{K} peers x {n_s:,} fp32 coords, {what} on torch CPU, {reps} reps in {el:.1f}s"}

    if rank == 0:
        line = {
            "metric": "aggregated peer-update GB/s (% HBM peak) at 1/2/4/8 MI355X",
            "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (device counter PRNG, SURVEY.md §8(d)); random-init model weights",
            "config": {"workload": f"{args.workload}: {rule} over {K} peers x {n:,} fp32 coords per GPU"
                                   + (" (cfg3 per-GPU tile; N=8 -> 1B coords)" if args.workload == "cfg3" else ""),
                       "rule": rule, "peers": K, "coords_per_gpu": n, "coords_total": n * world,
                       "parallelism": f"coord-shard x{world}" + (" + RCCL all-gather" if world > 1 else ""),
                       "pct_hbm_peak_step": round(4 * n * (K + 2) * world / step_s / 1e9 / world / HBM_PEAK_GBS, 4)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel_ms": round(kern_ms, 4), "alg_bytes_per_launch": alg_bytes},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
