#!/usr/bin/env python3
"""Benchmark of the aggregation hot path (driver contract: one JSON line).

Metric (BASELINE.json): aggregated peer-update GB/s (% HBM peak) at 1/2/4/8
MI355X.  value = peer-update bytes consumed by all ranks / step time.

Main line (default): cfg3's per-GPU coordinate tile -- FedAvg over 256 peers
x 125M fp32 coordinates PER GPU, resident in HBM (128 GB), weak scaling (at 8
GPUs the job is exactly cfg3, 1B coordinates x 256 peers).  A step = one
FedAvg pass (sum of K peers in list order, /K, w += 0.1*mean; reference
aggregator/aggregation.py:15-38) over the tile; at N > 1 each rank reduces its
round-robin coordinate chunks and an all-gather (RCCL over xGMI) reassembles
the global model, pipelined per chunk on a second stream.  Inputs are made on
device by the counter PRNG before timing; nothing is skipped inside the
timed region.

Sub-records (the "sub" object of the same line):
  cfg3_full     the FIXED cfg3 job, 1B coordinates x 256 peers (1.02 TB of
                peer data), as eight 125M-coordinate tiles: 8/N tiles per
                GPU, each tile's inputs regenerated outside the timed region
                (1.02 TB does not fit 288 GB); time = sum of tile kernel times
                + the all-gathers (reported separately).  Strong scaling.
  cfg2_dropin   cfg2 through the drop-in boundary: aggregate_models on a
                ResNet-18 state_dict (62 tensors, 11.7M params) x 64 updates
                -- the segment-table kernel the reference's caller reaches
  cfg4_median / cfg4_trimmed / median256 / trimmed256
                the robust rules at 128 peers x 100M and 256 peers x 100M
  cfg5          digest -> accept -> FedAvg over 256 serialized 100-MB updates
                (the GPU SHA-256 batch kernel; hashlib baseline beside it)
  delta         the trainer-side local update over 1B parameters
  inbox         16 serialized ResNet-18 updates landed in the device slab
                (vs the reference's pickle.loads), with the echo digest
                overlapped
  digest_flow   the reference's per-round 72 sign / verify digests through
                crypto.sign_data / verify_signature (vs 72 hashlib passes)
  broadcast     the global model's envelope pickled from the GPU (one D2H
                transfer) vs the reference's pickle of the CUDA state_dict
  cfg5_arrival  cfg5 as a node receives it: 256 x 100-MB messages in pinned
                receive buffers landed with host SHA-256 beside the DMAs,
                drop-in FedAvg over the accepted rows
(N = 1 only, except cfg3_full, which runs at every N.)

roofline.achieved = algorithmic bytes per launch 4n(K+2) / mean kernel time
(HIP events on the launch stream), peak 8.0 TB/s; roofline.traffic = HBM
bytes per launch from rocprofv3 PMC FETCH_SIZE/WRITE_SIZE
(profiles/traffic_<workload>.json, tools/pmc_traffic.py).
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time
import types

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from p2pdl_amd import ops, sharded  # noqa: E402

METRIC = "aggregated peer-update GB/s (% HBM peak) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0
W_PEER, UPD_SCALE, W_SCALE = 0xFFFFF, 1e-2, 5e-2
CFG3_COORDS, CFG3_TILE = 1_000_000_000, 125_000_000

WORKLOADS = {
    # name: (rule, peers, coords per GPU, seed)
    "cfg3": ("fedavg", 256, CFG3_TILE, 0x5EED0002),
    "cfg2": ("fedavg", 64, 11_689_512, 0x5EED0001),
    "cfg4-median": ("median", 128, 100_000_000, 0x5EED0003),
    "cfg4-trimmed": ("trimmed", 128, 100_000_000, 0x5EED0003),
    # north-star robust target: median over 256 peers (cfg3's K) on a 100M tile
    "median256": ("median", 256, 100_000_000, 0x5EED0005),
    "trimmed256": ("trimmed", 256, 100_000_000, 0x5EED0005),
    # K between the kernel families' sizes: the 4-lanes-per-coordinate LDS
    # kernels (K 129..255); not a BASELINE config, run on request only
    "median200": ("median", 200, 100_000_000, 0x5EED0009),
    "median160": ("median", 160, 100_000_000, 0x5EED0009),
    "trimmed200": ("trimmed", 200, 100_000_000, 0x5EED0009),
    "median96": ("median", 96, 100_000_000, 0x5EED000A),
    "trimmed96": ("trimmed", 96, 100_000_000, 0x5EED000A),
    "median24": ("median", 24, 100_000_000, 0x5EED000B),
    "trimmed24": ("trimmed", 24, 100_000_000, 0x5EED000B),
    "median32": ("median", 32, 100_000_000, 0x5EED000B),
    "trimmed32": ("trimmed", 32, 100_000_000, 0x5EED000B),
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
    # cfg2 through aggregate_models (ResNet-18 state_dict, segment kernel)
    "cfg2-dropin": ("dropin", 64, 11_689_512, 0x5EED0001),
    # land 16 serialized ResNet-18-sized updates (11.7M
    # params each) in the device slab vs the reference's pickle.loads
    "inbox": ("inbox", 16, 11_689_512, 0x5EED0007),
    # cfg5 as a node receives it: messages in pinned host buffers, digests on
    # the host beside the landing DMAs, FedAvg over the accepted slab rows
    "cfg5-arrival": ("arrival", 256, 25_000_000, 0x5EED0004),
    # the global model pickled for the broadcast
    "broadcast": ("broadcast", 1, 11_689_512, 0x5EED0008),
    # the reference's per-round digest work: 72 sign/verify hashes over 3 MLP
    # updates, through crypto.sign_data / verify_signature
    "digest-flow": ("digest-flow", 3, 535_818, 0),
}
SUB_N1 = ["cfg1", "cfg2-dropin", "cfg4-median", "cfg4-trimmed", "median256", "trimmed256", "cfg5", "delta", "inbox",
          "digest-flow", "broadcast", "cfg5-arrival"]
SUB_STEPS = {"cfg5": 2, "delta": 10, "inbox": 3, "digest-flow": 5, "broadcast": 5, "cfg5-arrival": 2}  # timed steps of the one-GPU sub-records
MSG_HEADER = 64  # bytes before the payload (keeps payloads 16-B aligned)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="cfg3", choices=sorted(WORKLOADS))
    ap.add_argument("--job", default="", choices=["", "cfg3-full"],
                    help="cfg3-full: the fixed 1B x 256 job as the main line (strong scaling)")
    ap.add_argument("--coords", type=int, default=0, help="override coordinates per GPU")
    ap.add_argument("--peers", type=int, default=0, help="override K")
    ap.add_argument("--chunks", type=int, default=8, help="all-gather pipeline chunks per rank (N>1)")
    ap.add_argument("--gather", default="overlap", choices=list(GATHER_LEGS),
                    help="N>1: each plane's all-gather on a second stream beside the next plane's reduction "
                         "(the product, sharded.PeerPlanes.aggregate_gather_), in line on the compute stream, "
                         "or p2p: overlapped, as a direct exchange (sharded.exchange_: grouped send/recv to "
                         "every peer at once); the default run also times the other legs (config.gather_legs)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--sub-cpu-seconds", type=float, default=6.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sub", action="store_true", help="main line only")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--no-reference-gpu", action="store_true",
                    help="skip timing the reference's torch ops on the GPU beside the product")
    return ap.parse_args()


class Ctx(types.SimpleNamespace):
    """world / rank / device / dist backend of this process."""


def cpu_record(res: dict, unit: str, kind: str, sample: str) -> dict:
    return {"value": round(res["value"], 3), "unit": unit, "cores": res["threads"], "kind": kind,
            "sample": sample, "value_1thread": round(res["value_1thread"], 3), "threads": res["threads"],
            "cpu_count": res["cpu_count"], "affinity": res["affinity"], "threads_rule": res["threads_rule"]}


def traffic_for(name: str, coords: int, peers: int):
    tfile = os.path.join(REPO, "profiles", f"traffic_{name}.json")
    if os.path.exists(tfile):
        with open(tfile) as f:
            tj = json.load(f)
        if tj.get("coords_per_launch") == coords and tj.get("peers") == peers:
            return tj.get("hbm_bytes_per_launch")
    return None


def roofline(alg_bytes: float, kern_ms: float, traffic, **extra) -> dict:
    ach = alg_bytes / (kern_ms / 1e3) / 1e9
    return dict({"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel_ms": round(kern_ms, 4),
                 "alg_bytes_per_launch": int(alg_bytes)}, **extra)


def dist_info() -> dict:
    """What ran the exchange: the process group's world size and backend,
    the RCCL version torch was built against, and the RCCL settings the
    environment gave it (NCCL_* / RCCL_*: channels, protocols, algorithms;
    empty = RCCL's own defaults, the build's channel policy)."""
    info = {"world_size": dist.get_world_size(), "backend": dist.get_backend(),
            "rccl_env": {k: v for k, v in sorted(os.environ.items())
                         if k.startswith(("NCCL_", "RCCL_")) and "SOCKET" not in k}}
    try:
        v = torch.cuda.nccl.version()
        info["rccl_version"] = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
    except Exception as e:  # noqa: BLE001 -- a record field, never fatal
        info["rccl_version"] = f"unknown ({type(e).__name__})"
    return info


def parallelism(c: Ctx) -> str:
    if c.world == 1:
        return "single GPU"
    via = "RCCL over xGMI" if c.backend == "nccl" else f"{c.backend} (rehearsal, ranks share one GPU)"
    return (f"coord-shard x{dist.get_world_size()} (process group world size, backend "
            f"{dist.get_backend()}), all_gather_into_tensor via {via}")


def oracle_expect(rule, K, m, seed, chunk=0, nranks=1, rank=0):
    """First m coordinates of a chunk-mapped workload, from the CPU oracle."""
    import oracle  # checker only

    peers = [oracle.synth(m, seed, p, UPD_SCALE, chunk, nranks, rank) for p in range(K)]
    w0 = oracle.synth(m, seed, W_PEER, W_SCALE, chunk, nranks, rank)
    rid = ops.rule_id(rule)
    if rid == 0:
        want, _ = oracle.fedavg(peers, w0)
    else:
        want, _ = oracle.robust(peers, rid, ops.trim_count(K) if rid == 2 else 0, w=w0)
    return want


def kernel_only_ms(fn, reps: int, stream=None) -> float:
    """Mean GPU time of the work ``fn`` enqueues, alone: the stream is kept
    busy by a spin kernel while the start event, the launch and the end event
    are queued behind it, so the host's launch overhead never shows between
    the events (for a ~5 us kernel it otherwise dominates)."""
    stream = stream or torch.cuda.current_stream()
    ev = []
    for _ in range(reps):
        torch.cuda._sleep(3_000_000)  # ~1.5 ms of spinning: the launch below is queued behind it
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        ev.append((e0, e1))
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in ev) / len(ev)


def bits_equal(a, b) -> bool:
    import numpy as np

    return np.array_equal(np.ascontiguousarray(a, dtype=np.float32).view(np.uint32),
                          np.ascontiguousarray(b, dtype=np.float32).view(np.uint32))


# ------------------------------------------------------------------ flat rules
PITCH = 64  # fp32 elements: every peer chunk starts a 256-B boundary


def pitched_slab(K, S, C, dev):
    """[K, S, C'] fp32 with C' = C rounded up to PITCH: peer p's chunk s is
    slab[p, s, :C], 256-B aligned like a separate allocation (a 16-B aligned
    chunk straddles one more 128-B HBM line per 4-KiB kernel tile)."""
    return torch.empty((K, S, -(-C // PITCH) * PITCH), dtype=torch.float32, device=dev)


# --gather legs: (exchange on a second stream?, sharded.EXCHANGES kind)
GATHER_LEGS = {"overlap": (True, "all_gather"), "inline": (False, "all_gather"), "p2p": (True, "p2p")}


def pipeline_summary(rank: int, kernel_ms, gather_ms, wall_ms: float, gather_bytes, world: int) -> dict:
    """One rank's reduce / all-gather pipeline over a step (or a job): the
    per-plane kernel and all-gather times (ms, HIP events on their own
    streams), the GPU wall time from the first kernel's start to the round's
    end, and the bytes each plane's all-gather writes (its output: every
    rank's piece).  overlap_frac = (sum kernel + sum gather - wall) / sum
    gather: 1 when every all-gather hid under the reductions, 0 when none did
    (in line), below 0 when time was lost between them.  algbw = output
    bytes / all-gather time (nccl-tests' convention), busbw = algbw (N-1)/N
    -- the bytes each rank received per second, the figure to hold against
    xGMI (one ring on one link: XGMI_LINK_GBS)."""
    ks, gs = float(sum(kernel_ms)), float(sum(gather_ms))
    alg = [b / (t / 1e3) / 1e9 for b, t in zip(gather_bytes, gather_ms) if t > 0]
    out = {"rank": int(rank), "kernel_ms": round(ks, 3), "allgather_ms": round(gs, 3), "wall_ms": round(wall_ms, 3),
           "overlap_frac": round((ks + gs - wall_ms) / gs, 4) if gs > 0 else None}
    if alg:
        mean = sum(alg) / len(alg)
        out.update({"allgather_algbw_gbs": round(mean, 2), "allgather_algbw_gbs_min": round(min(alg), 2),
                    "allgather_busbw_gbs": round(mean * (world - 1) / world, 2)})
    return out


def gather_verdict(rows) -> str:
    """What bounded the pipeline, from the per-rank summaries."""
    worst = max(rows, key=lambda r: r["wall_ms"])
    if worst["allgather_ms"] > worst["kernel_ms"]:
        return "all-gather bound (sum of all-gathers > sum of reductions on the slowest rank)"
    if (worst.get("overlap_frac") or 0) < 0.5:
        return "serialised (under half of the all-gather time hidden beside the reductions)"
    return "reduction bound (the all-gathers hide beside the reductions)"


def measure_flat(c: Ctx, args, name, rule, K, n, seed, steps, warmup, cpu_s, chunks, gather="overlap"):
    """Resident [K, n] slab per rank; a step = the rule over it (+ the chunked
    all-gather at N > 1).  Returns (record, ms_per_step)."""
    world, rank, dev = c.world, c.rank, c.dev
    # the product's memory-sharded layout (sharded.PeerPlanes): chunk-major
    # planes of K rows spanning <= 16 GB each, at least the all-gather
    # pipeline's chunks at N > 1
    # FedAvg: planes of whole split-kernel CU rounds and one short last plane
    # (sharded.round_plane_sizes; +1.3-1.7% on cfg3, same box) when that
    # gives the all-gather pipeline its chunks; else equal chunks
    sizes = (sharded.round_plane_sizes(
        K, n, torch.cuda.get_device_properties(dev).multi_processor_count * ops.SPLIT_TILE)
        if rule == "fedavg" and K >= 16 else [])
    if len(sizes) < (chunks if world > 1 else 1):
        S = sharded.plane_count(K, n, at_least=chunks if world > 1 else 1)
        sizes = [n // S] * S
    # C = the longest (first) plane: the synthetic chunk map's chunk (plane s
    # is generated as chunk s*N + rank of C; a shorter last plane as the head
    # of its chunk -- the all-gather places it at its own offset, round s
    # being N pieces of sizes[s])
    S, C = len(sizes), sizes[0]
    free, _ = torch.cuda.mem_get_info(dev)
    need = (K + 2 + world) * n * 4
    if need > free * 0.97:
        raise SystemExit(f"{name}: needs {need/1e9:.1f} GB, {free/1e9:.1f} GB free")
    log(f"[rank {rank}] {name}: generating {K} x {n:,} fp32 peer data ({K*n*4/1e9:.1f} GB) "
        f"as {plane_desc(K, sizes)}")
    planes, w = sharded.PeerPlanes(K, S, C, dev, sizes=sizes), pitched_slab(1, S, C, dev)[0]
    for s in range(S):  # local chunk s is global chunk s*N + rank
        for p in range(K):
            ops.fill_synthetic_(planes.row(s, p), seed, p, UPD_SCALE, C, world, rank + s * world)
        ops.fill_synthetic_(w[s, :sizes[s]], seed, W_PEER, W_SCALE, C, world, rank + s * world)
    w_full = torch.empty(n * world, dtype=torch.float32, device=dev) if world > 1 else None
    tables = planes.tables
    torch.cuda.synchronize()
    comp = torch.cuda.current_stream(dev)
    comm = torch.cuda.Stream(dev)
    kern = []

    gath, walls = [], []

    wviews = [w[s, :sizes[s]] for s in range(S)]

    def step(record=False):
        # the product's round (sharded.PeerPlanes.aggregate_gather_): every
        # plane reduced on the compute stream, its all-gather beside the next
        ev = {}

        def hook(s, phase, stream):
            e = torch.cuda.Event(enable_timing=True)
            e.record(stream)
            ev[(s, phase)] = e

        planes.aggregate_gather_(wviews, w_full, rule=rule, lr=0.1,
                                 comm=comm if world > 1 and GATHER_LEGS[gather][0] else None,
                                 hook=hook if record else None, exchange=GATHER_LEGS[gather][1])
        if record:
            end = torch.cuda.Event(enable_timing=True)
            end.record(comp)  # after the compute stream waited for the last all-gather
            walls.append((ev[(0, "reduce0")], end))
            for s in range(S):
                kern.append((ev[(s, "reduce0")], ev[(s, "reduce1")]))
                if world > 1:
                    gath.append((ev[(s, "gather0")], ev[(s, "gather1")]))

    # correctness spot check of the first warmup step: rank 0 checks the first
    # m coordinates of EVERY rank's first chunk, in its own w and, at N > 1,
    # where the all-gather placed them in the global model
    m = min(4096, C)
    check = not args.no_check and rank == 0
    for i in range(max(warmup, 1 if check else 0)):
        step()
        if i == 0 and check:
            torch.cuda.synchronize()
            bad = [g for g in range(world)
                   if not bits_equal((w_full[g * C:g * C + m] if world > 1 else w[0, :m]).cpu().numpy(),
                                     oracle_expect(rule, K, m, seed, C, world, g))]
            ml = min(m, sizes[-1])
            if S > 1 and not bits_equal(w[S - 1, :ml].cpu().numpy(),  # rank 0's last plane too
                                        oracle_expect(rule, K, ml, seed, C, world, (S - 1) * world)):
                bad.append(f"rank 0 plane {S - 1}")
            log(f"[rank 0] {name}: spot check vs oracle ({m} coords x {world} rank chunk(s)"
                f"{' + the last plane' if S > 1 else ''}): {'bit-exact' if not bad else f'MISMATCH on {bad}'}")
            if bad:
                raise SystemExit(f"bench: {name} output differs from the oracle")
        if world > 1:
            dist.barrier()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(record=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_ms = sum(a.elapsed_time(b) for a, b in kern) / len(kern)
    per_rank = None
    if world > 1:
        # every rank's pipeline per step (the diagnosis of a slow or stuck
        # rank: which side of the pipeline it lost time on, and how much of
        # the all-gather hid beside the reductions): per-plane kernel and
        # all-gather means over the timed steps, the GPU wall per step
        k_pl = [sum(kern[i * S + s][0].elapsed_time(kern[i * S + s][1]) for i in range(steps)) / steps
                for s in range(S)]
        g_pl = [sum(gath[i * S + s][0].elapsed_time(gath[i * S + s][1]) for i in range(steps)) / steps
                for s in range(S)]
        wall = sum(a.elapsed_time(b) for a, b in walls) / steps
        mine = torch.tensor([rank, wall] + k_pl + g_pl, dtype=torch.float64, device=dev)
        allr = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = []
        for t in (x.cpu().tolist() for x in allr):
            per_rank.append(pipeline_summary(int(t[0]), t[2:2 + S], t[2 + S:2 + 2 * S], t[1],
                                             [4 * sz * world for sz in sizes], world))
    ref_s = None
    if rule == "fedavg" and world == 1 and not args.no_reference_gpu:
        # the reference's aggregation loop (aggregator/aggregation.py:15-38) as a
        # node on this GPU runs it: torch ops over the same resident updates
        # (coordinate-wise, so chunk by chunk is the same computation)
        def reference_step():
            for s in range(S):
                ws = w[s, :sizes[s]]
                acc = torch.zeros_like(ws)  # :15
                for p in range(K):  # :25-28
                    acc += planes.row(s, p)
                acc /= K  # :31-32
                ws.add_(0.1 * acc)  # :36-38 (`+=` on the state_dict tensor)

        reference_step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(2):
            reference_step()
        torch.cuda.synchronize()
        ref_s = (time.perf_counter() - t0) / 2
    del planes, w, w_full, tables
    torch.cuda.empty_cache()
    step_s = elapsed / steps
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and cpu_s > 0:
        import oracle.cpu_baseline as cb  # baseline leg only

        if rule == "fedavg":
            n_s = 1_000_000
            res = cb.fedavg(K, n_s, cpu_s)
            what = "reference op sequence (aggregation.py:15-38)"
        elif rule == "median":
            n_s = 262_144
            res = cb.median(K, n_s, cpu_s)
            what = "torch.median(dim=0) (the build-defined rule on CPU)"
        else:
            n_s = 262_144
            res = cb.trimmed(K, n_s, ops.trim_count(K), cpu_s)
            what = "torch.sort(dim=0) + ascending sum of the kept ranks (the build-defined rule on CPU)"
        cpu = cpu_record(res, "GB/s", "port", f"{K} peers x {n_s:,} fp32 coords, {what}, "
                                              f"{res['reps']} reps in {res['seconds']}s")
    dtype = "fp32" if rule == "fedavg" else "fp32 (IEEE total order: f32 min/max/med3 networks, u32 keys for NaN tiles)"
    rec = {
        "workload": name, "value": round(K * n * 4 * world / step_s / 1e9, 2), "unit": "GB/s",
        "ms_per_step": round(step_s * 1e3, 4), "steps": steps, "scaling": "weak", "dtype": dtype,
        "config": {"workload": f"{name}: {rule} over {K} peers x {n:,} fp32 coords per GPU"
                               + (" (cfg3 per-GPU tile; N=8 -> the 1B-coordinate job)" if name == "cfg3" else ""),
                   "rule": rule, "peers": K, "coords_per_gpu": n, "coords_total": n * world,
                   "parallelism": parallelism(c),
                   "layout": f"{plane_desc(K, sizes)} (sharded.PeerPlanes), one launch per plane",
                   "pct_hbm_peak_step": round(4 * n * (K + 2) / step_s / 1e9 / HBM_PEAK_GBS, 4)}
                  | ({"per_rank": per_rank, "chunks_per_rank": S, "chunk_coords": C, "gather": gather,
                      "pipeline": gather_verdict(per_rank)} | dist_info() if per_rank else {})
                  | ({"reference_on_gpu_ms_per_step": round(ref_s * 1e3, 3),
                      "speedup_vs_reference_on_gpu": round(ref_s / step_s, 2)} if ref_s else {}),
        # per launch: the mean plane (= every plane when they are equal);
        # Σ bytes / Σ kernel time either way
        "roofline": roofline(4 * n * (K + 2) / S, kern_ms, traffic_for(name, n / S, K)),
        "cpu_baseline": cpu,
    }
    return rec, step_s


def plane_desc(K, sizes) -> str:
    runs = [(c, sizes.count(c)) for c in dict.fromkeys(sizes)]
    return (f"{len(sizes)} chunk-major plane(s): "
            + " + ".join(f"{cnt} x [{K} x {c:,}]" for c, cnt in runs))


# ------------------------------------------------------------------ cfg3 full job
def measure_cfg3_full(c: Ctx, args, passes=2, chunks=8, gather="overlap"):
    """The fixed cfg3 job: 1B coordinates x 256 peers (1.02 TB of peer data).
    Each rank works through its 1/N of the coordinates in tiles of 125M
    (128 GB of peer slices -- 1.02 TB does not fit 288 GB), global tile range
    [u*T*N, (u+1)*T*N) split round-robin by plane (round s = N pieces of the
    tile's plane s; planes of whole CU rounds, sharded.round_plane_sizes).  Per
    tile: regenerate the tile's 256 peer slices and w slice OUTSIDE the timed
    region, then reduce chunk by chunk on the compute stream while the
    all-gather of chunk s (RCCL over xGMI) runs on a second stream beside
    chunk s+1.  Reported time = sum over tiles of (first kernel start -> last
    all-gather end), max over ranks; the serial kernel and all-gather sums are
    reported beside it."""
    world, rank, dev = c.world, c.rank, c.dev
    K, seed, T = 256, WORKLOADS["cfg3"][3], CFG3_TILE
    C = T // chunks
    nchunks = CFG3_COORDS // C
    if nchunks % (world * chunks):
        raise SystemExit(f"cfg3-full: {nchunks} chunks do not split into tiles of {chunks} over {world} GPUs")
    per = nchunks // (world * chunks)  # tiles per rank
    # a tile's planes: whole split-kernel CU rounds + one short last plane
    # (sharded.round_plane_sizes, as the main line), else the 8 equal chunks
    sizes = sharded.round_plane_sizes(
        K, T, torch.cuda.get_device_properties(dev).multi_processor_count * ops.SPLIT_TILE)
    if len(sizes) < chunks:
        sizes = [C] * chunks
    S, M = len(sizes), sizes[0]
    planes, w = sharded.PeerPlanes(K, S, M, dev, sizes=sizes), pitched_slab(1, S, M, dev)[0]
    wviews = [w[s, :sizes[s]] for s in range(S)]
    w_full = torch.empty(CFG3_COORDS, dtype=torch.float32, device=dev) if world > 1 else None
    tables = planes.tables
    comp = torch.cuda.current_stream(dev)
    comm = torch.cuda.Stream(dev)
    wall, kern, gath, gpl = [], [], [], []
    checked = False
    for _ in range(passes):
        w_tot = k_tot = g_tot = 0.0
        g_pl = [0.0] * S
        for u in range(per):
            # plane s of tile u is generated as chunk (u*S + s)*N + rank of M
            # coordinates ("rank" r + u*S*N of an N-rank chunk map; a short
            # last plane as its head); round s's all-gather places the N
            # pieces of sizes[s] back to back inside the tile's global range
            vr = rank + u * S * world
            for s in range(S):
                for p in range(K):
                    ops.fill_synthetic_(planes.row(s, p), seed, p, UPD_SCALE, M, world, vr + s * world)
                ops.fill_synthetic_(w[s, :sizes[s]], seed, W_PEER, W_SCALE, M, world, vr + s * world)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            ev = {}

            def hook(s, phase, stream):
                e = torch.cuda.Event(enable_timing=True)
                e.record(stream)
                ev[(s, phase)] = e

            start = torch.cuda.Event(enable_timing=True)
            start.record(comp)
            # tile u is the global range [u*T*N, (u+1)*T*N)
            tile_full = w_full[u * T * world:(u + 1) * T * world] if world > 1 else None
            planes.aggregate_gather_(wviews, tile_full, rule="fedavg", lr=0.1,
                                     comm=comm if world > 1 and GATHER_LEGS[gather][0] else None, hook=hook,
                                     exchange=GATHER_LEGS[gather][1])
            end = torch.cuda.Event(enable_timing=True)
            end.record(comp)
            torch.cuda.synchronize()
            w_tot += start.elapsed_time(end)
            k_tot += sum(ev[(s, "reduce0")].elapsed_time(ev[(s, "reduce1")]) for s in range(S))
            if world > 1:
                for s in range(S):
                    g_pl[s] += ev[(s, "gather0")].elapsed_time(ev[(s, "gather1")])
                g_tot = sum(g_pl)
            if not checked and not args.no_check and rank == 0:
                m = 4096
                got = (w_full[:m] if world > 1 else w[0, :m]).cpu().numpy()  # global chunk 0: rank 0, tile 0
                ok = bits_equal(got, oracle_expect("fedavg", K, m, seed, M, world, 0))
                log(f"[rank 0] cfg3-full: spot check of global chunk 0 vs oracle: {'bit-exact' if ok else 'MISMATCH'}")
                if not ok:
                    raise SystemExit("bench: cfg3-full differs from the oracle")
                checked = True
        wall.append(w_tot)
        kern.append(k_tot)
        gath.append(g_tot)
        gpl.append(g_pl)
    best = min(range(passes), key=lambda i: wall[i])  # best pass (each pass is the whole job)
    tot, k_ms, g_ms = wall[best], kern[best], gath[best]
    per_rank = None
    if world > 1:
        mine = torch.tensor([rank, tot, k_ms] + gpl[best], dtype=torch.float64, device=dev)
        allr = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        rows = [x.cpu().tolist() for x in allr]
        # per plane: the job's all-gathers of that plane summed over its tiles
        # (each writes 4 * sizes[s] * N bytes per tile)
        per_rank = []
        for r in rows:
            d = pipeline_summary(int(r[0]), [r[2]], r[3:3 + S], r[1], [4 * sz * world * per for sz in sizes], world)
            d["kernel_ms_sum"], d["allgather_ms_sum"], d["ms_per_job"] = d.pop("kernel_ms"), d.pop("allgather_ms"), \
                d.pop("wall_ms")
            per_rank.append(d)
        tot, k_ms = (max(r[i] for r in rows) for i in (1, 2))
        g_ms = max(sum(r[3:3 + S]) for r in rows)
    del planes, w, w_full, tables
    torch.cuda.empty_cache()
    peer_bytes = K * CFG3_COORDS * 4
    return {
        "workload": "cfg3_full", "value": round(peer_bytes / (tot / 1e3) / 1e9, 2), "unit": "GB/s",
        "ms_per_job": round(tot, 3), "kernel_ms_sum": round(k_ms, 3), "allgather_ms_sum": round(g_ms, 3),
        "scaling": "strong", "dtype": "fp32",
        "config": {"workload": f"cfg3 full job: fedavg over {K} peers x {CFG3_COORDS:,} fp32 coords "
                               f"({peer_bytes/1e12:.3f} TB); {per} tile(s) of {T:,} coords per GPU, "
                               f"{plane_desc(K, sizes)} per tile", "tiles_per_gpu": per,
                   "parallelism": parallelism(c)}
                  | ({"per_rank": per_rank, "gather": gather,
                      "pipeline": gather_verdict([{"wall_ms": r["ms_per_job"], "kernel_ms": r["kernel_ms_sum"],
                                                   "allgather_ms": r["allgather_ms_sum"],
                                                   "overlap_frac": r["overlap_frac"]} for r in per_rank])}
                     | dist_info() if per_rank else {}) | {
                   "timing": "sum over tiles of first-kernel-start -> last-all-gather-end (HIP events; "
                             "all-gather of chunk s overlapped with chunk s+1); inputs regenerated per tile "
                             "outside the timed region (1.02 TB > 288 GB HBM)"},
        "roofline": roofline(4 * T * (K + 2) / S, k_ms / (per * S), traffic_for("cfg3-chunk", T / S, K)),
    }


# ------------------------------------------------------------------ drop-in (cfg1 / cfg2)
MLP_SHAPES = [("fc1.weight", (512, 784)), ("fc1.bias", (512,)), ("fc2.weight", (256, 512)),
              ("fc2.bias", (256,)), ("fc3.weight", (10, 256)), ("fc3.bias", (10,))]  # models/model.py:6-8


def resnet18_param_shapes():
    """The 62 parameter tensors of torchvision's ResNet-18 (11,689,512 fp32)."""
    shapes = [("conv1.weight", (64, 3, 7, 7)), ("bn1.weight", (64,)), ("bn1.bias", (64,))]
    cin = 64
    for li, cout in enumerate((64, 128, 256, 512), start=1):
        for blk in range(2):
            p = f"layer{li}.{blk}."
            c0 = cin if blk == 0 else cout
            shapes += [(p + "conv1.weight", (cout, c0, 3, 3)), (p + "bn1.weight", (cout,)), (p + "bn1.bias", (cout,)),
                       (p + "conv2.weight", (cout, cout, 3, 3)), (p + "bn2.weight", (cout,)), (p + "bn2.bias", (cout,))]
            if blk == 0 and cin != cout:
                shapes += [(p + "downsample.0.weight", (cout, cin, 1, 1)), (p + "downsample.1.weight", (cout,)),
                           (p + "downsample.1.bias", (cout,))]
        cin = cout
    return shapes + [("fc.weight", (1000, 512)), ("fc.bias", (1000,))]


def _numel(shape):
    out = 1
    for s in shape:
        out *= s
    return out


def reference_on_gpu(model, updates, K, steps, warmup):
    """Seconds per call of the reference's aggregation loop (reference
    aggregator/aggregation.py:15-38, restated op for op) on the GPU tensors
    of `model` and the update dicts: what the deployed reference -- model on
    cuda, node/node.py:28-29 -- costs on this box.  Modifies the model."""
    received = [{"model": u} for u in updates]

    def call():
        accumulated_updates = {key: torch.zeros_like(param) for key, param in model.state_dict().items()}  # :15
        for received_model in received:  # :25-28
            local_update = received_model["model"]
            for key in accumulated_updates:
                accumulated_updates[key] += local_update[key]
        for key in accumulated_updates:  # :31-32
            accumulated_updates[key] /= K
        learning_rate = 0.1
        for key in model.state_dict():  # :36-38
            model.state_dict()[key] += learning_rate * accumulated_updates[key]

    with torch.no_grad():
        for _ in range(max(warmup, 1)):
            call()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            call()
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def measure_dropin(c: Ctx, args, name, K, seed, steps, warmup, cpu_s):
    """aggregate_models (reference aggregator/aggregation.py:7-46) on a fake
    Node, end to end: host segment table + one kernel launch per call.
    Updates are rows of a [K, N] device slab, as DeviceInbox lands them."""
    from p2pdl_amd.aggregator import aggregation as agg

    dev = c.dev
    shapes = MLP_SHAPES if name == "cfg1" else resnet18_param_shapes()
    sizes = [_numel(s) for _, s in shapes]
    n = sum(sizes)
    offs = [0]
    for sz in sizes:
        offs.append(offs[-1] + sz)
    model = torch.nn.Module()
    for i, (nm, shape) in enumerate(shapes):
        model.register_parameter(nm.replace(".", "__"), torch.nn.Parameter(
            torch.empty(shape, dtype=torch.float32, device=dev), requires_grad=False))
    flat_w = torch.empty(n, dtype=torch.float32, device=dev)
    ops.fill_synthetic_(flat_w, seed, W_PEER, W_SCALE)
    with torch.no_grad():
        for i, p in enumerate(model.parameters()):
            p.view(-1).copy_(flat_w[offs[i]:offs[i + 1]])
    # the updates live where DeviceInbox lands received updates: rows of one
    # [K, N'] slab (tensors at 256-B aligned offsets), generated on device
    from p2pdl_amd.node.inbox import DeviceInbox

    inbox = DeviceInbox(model.state_dict(), k_max=K, device=dev)
    slab = inbox.slab
    for p in range(K):
        ops.fill_synthetic_(slab[p], seed, p, UPD_SCALE)
    landed = [inbox.view(j) for j in range(K)]
    keys = [nm.replace(".", "__") for nm, _ in shapes]
    assert inbox.layout[keys[0]][0] == 0 and sizes[0] >= 4096  # the spot check's coordinates
    # the general path's updates: plain dicts whose every tensor is its own
    # allocation, as pickle.loads hands them to the reference's listener
    # (node/node.py:138-141); the same values as the slab rows
    plain = [{k: slab[j, inbox.layout[k][0]:inbox.layout[k][0] + sizes[i]].view(shapes[i][1]).clone()
              for i, k in enumerate(keys)} for j in range(K)]
    updates = landed
    node = types.SimpleNamespace(model=model, trainers_list=[0] * K, addr="127.0.0.1", port=1, neighbors=[],
                                 received_models=[])
    saved = agg.broadcast_global_model_update
    agg.broadcast_global_model_update = lambda self: None  # networking is out of scope
    comp = torch.cuda.current_stream(dev)
    ev = []

    def call(record=False):
        node.received_models.extend({"model": u, "sender": j} for j, u in enumerate(updates))
        if record:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(comp)
        agg.aggregate_models(node)
        if record:
            e1.record(comp)
            ev.append((e0, e1))

    def timed_calls():
        # host wall time per call, the same way for both paths: no events
        # inside the timed loop (the kernel is timed in a separate pass)
        for _ in range(max(warmup, 2)):
            call()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            call()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps

    try:
        call()
        torch.cuda.synchronize()
        if not args.no_check:
            import oracle  # checker only

            m = min(n, 4096)
            got = torch.cat([p.detach().reshape(-1) for p in model.parameters()])[:m].cpu().numpy()
            want, _ = oracle.fedavg([oracle.synth(m, seed, p, UPD_SCALE) for p in range(K)],
                                    oracle.synth(m, seed, W_PEER, W_SCALE))
            ok = bits_equal(got, want)
            log(f"{name}: drop-in spot check vs oracle ({m} coords): {'bit-exact' if ok else 'MISMATCH'}")
            if not ok:
                raise SystemExit(f"bench: {name} drop-in differs from the oracle")
        step_s = timed_calls()
        for _ in range(steps):  # the kernel (+ table) time, HIP events around each call
            call(record=True)
        torch.cuda.synchronize()
        ev_fast = list(ev)
        # the kernel alone: the launch aggregate_models cached on the
        # validated model-state entry (ops.relaunch: no table work), queued
        # behind a spin so no host time falls between the events
        from p2pdl_amd.aggregator.model_state import model_state

        keys_m, ws_m, st_m = model_state(model)
        launch = st_m.extra.get("launch") if st_m is not None else None
        kernel_path = (("split kernel over the slab rows as flat peers (ops._rows_entry)"
                        if launch[2][5][0] == "rows" else "VGPR segment kernel (+ split tiles when planned)")
                       if launch is not None else "general path")
        kernel_ms = None
        if launch is not None:
            kernel_ms = kernel_only_ms(lambda: ops.relaunch(launch[2], dev, len(ws_m), K, 0.1), steps, comp)
        # the general path (plain dicts of tensors, e.g. from pickle.loads):
        # the peer table gathered in C from the L x K update tensors
        updates = plain
        general_s = timed_calls()
        ev.clear()
        # the general path's launch alone (its cached table, ops.relaunch),
        # and its host wall time with a new table every call (a round whose
        # updates arrive at new addresses: the C gather, the chunk list, H2D)
        gen_entry = next(reversed(ops._TABLES.values()))
        general_kernel_ms = kernel_only_ms(lambda: ops.relaunch(gen_entry, dev, len(keys), K, 0.1), steps, comp)
        general_route = gen_entry[5][2][3] if gen_entry[5][0] != "rows" and gen_entry[5][2] else "vgpr"
        # the same route over the slab rows' own views (the landed bytes, one
        # allocation): what the kernel reads there against the per-tensor
        # allocations above is where the caller's allocator put the tensors
        # (UTCL1 translation misses), not the kernel
        import numpy as np

        vptrs = np.array([[slab[j].data_ptr() + 4 * inbox.layout[k][0] for j in range(K)] for k in keys_m],
                         dtype=np.uint64)
        ops.aggregate_ptr_table_(ws_m, vptrs, "fedavg")
        v_entry = next(reversed(ops._TABLES.values()))
        views_route = v_entry[5][2][3] if v_entry[5][0] != "rows" and v_entry[5][2] else "vgpr"
        views_kernel_ms = kernel_only_ms(lambda: ops.relaunch(v_entry, dev, len(keys), K, 0.1), steps, comp)
        fresh = []
        for _ in range(steps):
            ops._TABLES.clear()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            call()
            torch.cuda.synchronize()
            fresh.append(time.perf_counter() - t0)
        general_fresh_s = sorted(fresh)[len(fresh) // 2]
        ref_s = None if args.no_reference_gpu else reference_on_gpu(model, plain, K, steps, warmup)
    finally:
        agg.broadcast_global_model_update = saved
    call_ms = sum(a.elapsed_time(b) for a, b in ev_fast) / len(ev_fast)
    # the same byte count through the flat C-ABI kernel (one buffer per peer), for comparison
    table = ops.pointer_table([slab[p, :n] for p in range(K)], dev)
    fe = []
    for i in range(steps + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(comp)
        ops.aggregate(None, "fedavg", w=flat_w, lr=0.1, table=table)
        e1.record(comp)
        if i >= 2:
            fe.append((e0, e1))
    torch.cuda.synchronize()
    flat_ms = sum(a.elapsed_time(b) for a, b in fe) / len(fe)
    del slab, flat_w, table, updates, model, inbox, landed, plain
    torch.cuda.empty_cache()
    cpu = None
    if not args.no_cpu_baseline and cpu_s > 0:
        import oracle.cpu_baseline as cb  # baseline leg only

        res = cb.fedavg_state_dict(K, sizes, cpu_s, seed)
        cpu = cpu_record(res, "GB/s", "port", f"{len(sizes)}-tensor state_dict ({n:,} params) x {K} updates, "
                                              f"reference per-key op sequence (aggregation.py:15-38) on torch "
                                              f"CPU, {res['reps']} reps in {res['seconds']}s")
        # the same calls as microseconds per aggregate_models call (cfg1 is latency-bound)
        cpu["us_per_call"] = round(4.0 * K * n / (res["value"] * 1e9) * 1e6, 1)
        cpu["us_per_call_1thread"] = round(4.0 * K * n / (res["value_1thread"] * 1e9) * 1e6, 1)
    return {
        "workload": name.replace("-", "_"), "value": round(K * n * 4 / step_s / 1e9, 2), "unit": "GB/s",
        "ms_per_step": round(step_s * 1e3, 4), "us_per_call": round(step_s * 1e6, 1),
        "us_per_call_general_path": round(general_s * 1e6, 1), "steps": steps,
        "general_path": {
            "what": "plain dicts of separately allocated tensors (pickle.loads' form, node/node.py:138-141): "
                    "the C-gathered peer table, route " + general_route,
            "route": general_route, "us_per_call": round(general_s * 1e6, 1),
            "us_per_call_new_table_every_call": round(general_fresh_s * 1e6, 1),
            "kernel_ms": round(general_kernel_ms, 4),
            "frac_of_hbm_peak": round(4 * n * (K + 2) / (general_kernel_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "same_route_over_slab_views": {
                "route": views_route, "kernel_ms": round(views_kernel_ms, 4),
                "frac_of_hbm_peak": round(4 * n * (K + 2) / (views_kernel_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                "what": "the general path's table built over the DeviceInbox slab rows' own views (one "
                        "allocation) instead of per-tensor clones: the kernel's rate without the clones' "
                        "address-translation misses"}},
        "reference_on_gpu": None if ref_s is None else {
            "us_per_call": round(ref_s * 1e6, 1), "speedup": round(ref_s / step_s, 1),
            "what": "the reference's aggregate_models loop (aggregation.py:15-38) as a node on this GPU runs "
                    "it: torch ops on the cuda tensors, state_dict() rebuilt per key at :37-38; same model "
                    "and updates (plain dicts)"},
        "scaling": "weak", "dtype": "fp32",
        "config": {"workload": f"{name}: drop-in aggregate_models, {len(sizes)}-tensor state_dict "
                               f"({n:,} params) x {K} updates landed in a DeviceInbox slab, one "
                               f"segment-table launch per call",
                   "peers": K, "coords_per_gpu": n, "tensors": len(sizes), "parallelism": "single GPU",
                   "us_per_call": round(step_s * 1e6, 1), "us_per_call_general_path": round(general_s * 1e6, 1)}
                  | ({"reference_on_gpu_us_per_call": round(ref_s * 1e6, 1),
                      "speedup_vs_reference_on_gpu": round(ref_s / step_s, 1)} if ref_s else {}),
        "roofline": roofline(4 * n * (K + 2), kernel_ms or call_ms, traffic_for(name, n, K),
                             kernel_path=kernel_path,
                             timing=("the kernel alone: HIP events around the cached launch "
                                     "(ops.relaunch) queued behind a spin kernel; call_ms: events around the "
                                     "whole aggregate_models call; value / us_per_call: host wall time, no events"
                                     if kernel_ms else "HIP events around aggregate_models (no cached launch)"),
                             call_ms=round(call_ms, 4),
                             flat_kernel_ms=round(flat_ms, 4),
                             vs_flat_kernel=round(flat_ms / (kernel_ms or call_ms), 4)),
        "cpu_baseline": cpu,
    }


# ------------------------------------------------------------------ digest (cfg5 / sha256)
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
    ptrs = torch.tensor([buf.data_ptr() + o for o in offsets], dtype=torch.int64, device=dev)
    lens_d = torch.tensor([msg_bytes] * K, dtype=torch.int64, device=dev)
    digests = torch.empty((K, 32), dtype=torch.uint8, device=dev)
    lib = ops.N.lib()

    def digest_gpu():
        ops.N.check(lib.p2p_sha256_batch(ptrs.data_ptr(), lens_d.data_ptr(), K, digests.data_ptr(),
                                         ops.N.stream_handle()), "sha256")

    from p2pdl_amd.utils import digests as dg

    lens_h = [msg_bytes] * K
    host_route = not (K >= dg.GPU_BATCH_MIN and msg_bytes <= dg.GPU_MAX_MESSAGE)

    def digest():
        # the product's route for device-resident messages (utils/digests.py
        # digest_device_messages): these long messages hash on the host threads
        # with the D2H beside them; the GPU batch kernel is timed apart below
        digests.copy_(dg.digest_device_messages(buf, offsets, lens_h))

    digest_gpu()
    expected = digests.clone()  # what the senders signed (untimed)
    torch.cuda.synchronize()
    g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g0.record()
    digest_gpu()  # the GPU batch kernel alone, for the record
    g1.record()
    torch.cuda.synchronize()
    gpu_kernel_ms = g0.elapsed_time(g1)
    digest()
    torch.cuda.synchronize()
    assert torch.equal(digests, expected), "host route digests differ from the GPU kernel's"
    for p in (0, K - 1):  # cross-check two digests on the host (checker only)
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
    step_s = (time.perf_counter() - t0) / args.steps
    sha_ms = sum(a.elapsed_time(b) for a, b, _ in kern) / len(kern)
    agg_ms = sum(b.elapsed_time(c) for _, b, c in kern) / len(kern)
    hashed = K * msg_bytes
    acc = K - len(bad)
    agg_bytes = 4 * n * (acc + 2) if rule == "fused" else 0
    d2h_gbs = sha_host = None
    if host_route:
        # the host route's two ceilings on this box: pinned device-to-host
        # copies over PCIe, and the hashing threads over the same K
        # full-length messages from pinned host memory (the first
        # hash_threads() messages copied out once, hashed in turn)
        d2h_gbs = pinned_copy_gbs(dev, to_device=False)
        pins = []
        for p in range(min(K, dg.hash_threads())):
            pins.append(torch.empty(msg_bytes, dtype=torch.uint8, pin_memory=True))
            pins[-1].copy_(buf[offsets[p]:offsets[p] + msg_bytes])
        sha_host = host_sha_ceiling([memoryview(t.numpy()) for t in pins], K)
        del pins
    cpu = None
    if not args.no_cpu_baseline:
        import oracle.cpu_baseline as cb  # baseline leg only

        sample = [bytes(buf[offsets[p]:offsets[p] + min(msg_bytes, 16 << 20)].cpu().numpy()) for p in range(min(K, 64))]
        res = cb.sha256(sample, args.cpu_seconds)
        what = (f"hashlib.sha256 (OpenSSL, the function behind reference utils/crypto.py:56) over "
                f"{len(sample)} x {len(sample[0]):,} B")
        if rule == "fused":
            # end to end on the host: hash every message, then the reference's
            # FedAvg op sequence over the accepted payloads (GB/s of hashed bytes)
            fed = cb.fedavg(acc, 1_000_000, max(2.0, args.cpu_seconds / 3))
            host_s = hashed / (res["value"] * 1e9) + agg_bytes / 4 / (acc + 2) * acc / (fed["value"] * 1e9)
            res = dict(res, value=hashed / host_s / 1e9, value_1thread=res["value_1thread"])
            what += f" + reference FedAvg ops over {acc} accepted (host, {fed['value']:.1f} GB/s)"
        cpu = cpu_record(res, "GB/s", "port", f"{what}, {res['reps']} reps in {res['seconds']}s")
    del buf, ptrs, lens_d, digests, expected, payload_tbl, w
    torch.cuda.empty_cache()
    return {
        "workload": args.workload, "value": round(hashed / step_s / 1e9, 3), "unit": "GB/s", "steps": args.steps,
        "ms_per_step": round(step_s * 1e3, 3), "scaling": "weak", "dtype": "u32 (SHA-256) + fp32",
        "data": "synthetic serialized updates (64-B header + device-PRNG fp32 payload)",
        "config": {"workload": f"{args.workload}: {K} messages x {msg_bytes:,} B"
                               + (f", {len(bad)} corrupted, FedAvg over {acc} accepted" if rule == "fused" else ""),
                   "peers": K, "coords_per_peer": n, "parallelism": "single GPU (replicas only)",
                   "hash_threads": dg.hash_threads() if host_route else None},
        "roofline": cfg5_roofline(host_route, hashed, step_s, sha_ms, agg_ms, agg_bytes, gpu_kernel_ms, K,
                                  sha_host, d2h_gbs),
        "cpu_baseline": cpu,
    }


def host_sha_ceiling(views, K: int) -> float:
    """GB/s the product's hashing threads reach on this box over K
    full-length messages already in pinned host memory, with nothing else
    running: utils/digests.py's own pool (hash_threads() threads) hashing
    views[p % len(views)] for p < K -- the same lengths, count and threads as
    the step, with no PCIe copy to wait on.  The best of two passes.  The
    host route's digest leg cannot beat it."""
    import hashlib

    from p2pdl_amd.utils import digests as dg

    pool = dg.hash_pool()
    total = float(sum(len(views[p % len(views)]) for p in range(K)))
    best = None
    for _ in range(2):
        t0 = time.perf_counter()
        list(pool.map(lambda p: hashlib.sha256(views[p % len(views)]).digest(), range(K)))
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return total / best / 1e9


def pinned_copy_gbs(dev, to_device: bool, nbytes: int = 1 << 30) -> float:
    """Pinned host <-> device copy rate over PCIe (GB/s), best of 3."""
    pin = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    best = None
    for _ in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        (d.copy_(pin, non_blocking=True) if to_device else pin.copy_(d, non_blocking=True))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    del pin, d
    return nbytes / best / 1e9


def cfg5_roofline(host_route, hashed, step_s, sha_ms, agg_ms, agg_bytes, gpu_kernel_ms, K, sha_host, d2h_gbs):
    """cfg5's bound, labelled by what runs.  These long
    messages hash on the host (utils/digests.py digest_device_messages: each
    message streamed over PCIe D2H to a SHA-NI thread), so the digest leg is
    bounded by min(this box's hashlib rate on the same threads, the pinned D2H
    rate) and carries no kernel time or HBM fraction; the HBM fraction
    belongs to the FedAvg kernel leg alone.  The SHA-256 batch kernel is
    timed beside it for the record (a serial chain per message)."""
    # serial-chain issue bound of the batch kernel: one wave issues ~1
    # instruction / 4 cycles at 2.4 GHz, ~910 instructions per 64-B block
    chain = round(min(K, 65536) * 64 / (910 * 4 / 2.4e9) / 1e9, 2)
    kernel = {"sha256_kernel_ms": round(gpu_kernel_ms, 3),
              "sha256_kernel_gbs": round(hashed / (gpu_kernel_ms / 1e3) / 1e9, 2),
              "sha256_chain_issue_bound_gbs": chain}
    fed = {"fedavg_kernel_ms": round(agg_ms, 3),
           "fedavg_gbs": round(agg_bytes / (agg_ms / 1e3) / 1e9, 1) if agg_bytes else None,
           "fedavg_frac_of_hbm_peak": round(agg_bytes / (agg_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if agg_bytes else None}
    achieved = hashed / step_s / 1e9  # end to end: digest + accept + FedAvg
    if host_route:
        peaks = [x for x in (sha_host, d2h_gbs) if x]
        peak = min(peaks) if peaks else None
        return {"bound": "host-sha256 / pcie-d2h (digest on host SHA-NI threads; no kernel)",
                "achieved": round(achieved, 2), "peak": round(peak, 2) if peak else None, "unit": "GB/s",
                "frac": round(achieved / peak, 3) if peak else None, "traffic": None,
                "digest_route": "host", "digest_ms": round(sha_ms, 3),
                "host_sha_bound_gbs": round(sha_host, 2) if sha_host else None,
                "pcie_d2h_gbs": round(d2h_gbs, 2) if d2h_gbs else None,
                "peak_what": "min(the product's hashing pool over the same K full-length messages from pinned "
                             "host memory, no copies beside it; pinned D2H over PCIe), both measured on this box "
                             "in this run"} | fed | kernel
    return {"bound": "int-alu (serial SHA-256 chain per message; DESIGN.md K3)",
            "achieved": round(hashed / (sha_ms / 1e3) / 1e9, 2), "peak": chain, "unit": "GB/s",
            "frac": round(hashed / (sha_ms / 1e3) / 1e9 / chain, 3), "traffic": None,
            "digest_route": "gpu", "kernel_ms": round(sha_ms, 3)} | fed | kernel


def run_cfg5_arrival(args, K, n, seed, dev):
    """cfg5 as a node receives it: K serialized updates ({'w': n fp32},
    pickled like node/node.py:285) in the inbox's pinned receive buffers.
    A step lands every message (one DMA + the landing kernel each) with its
    SHA-256 on the host hashing threads beside the DMAs
    (DeviceInbox.land(..., digest=True)), accepts the updates whose digest
    matches what the sender signed, and runs the drop-in aggregate_models
    (FedAvg) over the accepted slab rows.  The digest cache is emptied before
    every step, so every message is hashed in every step.  value = hashed
    bytes per second, as for cfg5."""
    import hashlib
    import pickle

    import numpy as np

    from p2pdl_amd.aggregator import aggregation as agg
    from p2pdl_amd.node.inbox import DeviceInbox
    from p2pdl_amd.utils import digests

    from p2pdl_amd.node.inbox import ZeroCopyParser

    proto = pickle.dumps({"w": torch.zeros(n)})
    data = ZeroCopyParser(proto).parse()["w"].storage.data  # the payload's window of proto
    pay = np.frombuffer(data, dtype=np.uint8).ctypes.data - np.frombuffer(proto, dtype=np.uint8).ctypes.data
    assert len(data) == 4 * n and proto[pay:pay + 4 * n] == bytes(4 * n)
    del data
    nbytes = len(proto)
    template = {"w": torch.empty(n, dtype=torch.float32, device=dev)}
    inbox = DeviceInbox(template, k_max=K, device=dev, max_message_bytes=nbytes,
                        pool_bytes=(K + 1) * nbytes)
    log(f"cfg5-arrival: {K} pinned messages of {nbytes:,} B ({K * nbytes / 1e9:.1f} GB)")
    stage = torch.empty(n, dtype=torch.float32, device=dev)
    msgs, expected = [], []
    for p in range(K):
        m = inbox.message_buffer(nbytes)
        m.buf[:pay].copy_(torch.frombuffer(bytearray(proto[:pay]), dtype=torch.uint8))
        m.buf[pay + 4 * n:nbytes].copy_(torch.frombuffer(bytearray(proto[pay + 4 * n:]), dtype=torch.uint8))
        ops.fill_synthetic_(stage, seed, p, UPD_SCALE)
        m.buf[pay:pay + 4 * n].copy_(stage.view(torch.uint8))
        msgs.append(m)
    torch.cuda.synchronize()
    pool = digests.hash_pool()
    expected = list(pool.map(lambda m: hashlib.sha256(m.view()).digest(), msgs))  # what the senders signed
    bad = [p for p in range(K) if (p * 7919) % 10 == 3]  # ~10% corrupted in flight, as cfg5
    for p in bad:
        msgs[p].buf[pay + 4000] ^= 0x40
    w0 = torch.empty(n, dtype=torch.float32, device=dev)
    ops.fill_synthetic_(w0, seed, W_PEER, W_SCALE)
    model = torch.nn.Module()
    model.register_parameter("w", torch.nn.Parameter(w0.clone(), requires_grad=False))
    node = types.SimpleNamespace(model=model, trainers_list=[], addr="127.0.0.1", port=1, neighbors=[],
                                 received_models=[])
    saved = agg.broadcast_global_model_update
    agg.broadcast_global_model_update = lambda self: None

    def step():
        inbox.reset()
        landed = [inbox.land(m, digest=True) for m in msgs]
        ok = [inbox.digest(k) == expected[k] for k in range(K)]
        node.received_models[:] = [{"model": u, "sender": k} for k, u in enumerate(landed) if ok[k]]
        agg.aggregate_models(node)
        torch.cuda.synchronize()
        return ok

    try:
        times = []
        for i in range(max(args.warmup, 1) + args.steps):
            with torch.no_grad():
                model.w.copy_(w0)
            digests.CACHE.clear()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ok = step()
            dt = time.perf_counter() - t0
            if i >= max(args.warmup, 1):
                times.append(dt)
            if i == 0:
                acc = [p for p in range(K) if ok[p]]
                if acc != [p for p in range(K) if p not in bad]:
                    raise SystemExit("bench: cfg5-arrival accepted the wrong updates")
                if not args.no_check:
                    import oracle  # checker only

                    m_ = 4096
                    want, _ = oracle.fedavg([oracle.synth(m_, seed, p, UPD_SCALE) for p in acc],
                                            oracle.synth(m_, seed, W_PEER, W_SCALE))
                    good = bits_equal(model.w[:m_].cpu().numpy(), want)
                    log(f"cfg5-arrival: {len(acc)} accepted, FedAvg spot check vs oracle: "
                        f"{'bit-exact' if good else 'MISMATCH'}")
                    if not good:
                        raise SystemExit("bench: cfg5-arrival FedAvg differs from the oracle")
    finally:
        agg.broadcast_global_model_update = saved
        digests.CACHE.clear()
    step_s = min(times)
    hashed = K * nbytes
    # the step's two ceilings on this box: the hashing pool over these same
    # pinned messages with nothing beside it, and pinned H2D over PCIe (every
    # message crosses once; the two run concurrently in the step)
    sha_gbs = host_sha_ceiling([m.view() for m in msgs], K)
    h2d_gbs = pinned_copy_gbs(dev, to_device=True)
    bound = min(sha_gbs, h2d_gbs)
    cpu = None
    if not args.no_cpu_baseline:
        import oracle.cpu_baseline as cb  # baseline leg only

        ks = min(K, 16)  # a bounded sample: the first 16 messages (2 of them corrupted)
        sample = [bytes(msgs[p].view()) for p in range(ks)]
        res = cb.arrival(sample, expected[:ks], w0.cpu(), args.cpu_seconds)
        cpu = cpu_record(res, "GB/s", "port",
                         f"{ks} of the {K} messages ({nbytes:,} B each, {ks - res['accepted']} corrupted): hashlib "
                         f"SHA-256 of each on a thread pool (utils/crypto.py:56), pickle.loads of the "
                         f"{res['accepted']} that match (node/node.py:138) and the reference's FedAvg ops over them "
                         f"(aggregation.py:15-38) on torch CPU; {res['reps']} reps in {res['seconds']}s")
        del sample
    for m in msgs:
        m.release()
    del inbox, msgs, model, w0, stage, template, node
    import gc

    gc.collect()  # the inbox and its pinned buffers refer to each other
    torch.cuda.empty_cache()
    return {
        "workload": "cfg5_arrival", "value": round(hashed / step_s / 1e9, 3), "unit": "GB/s", "steps": args.steps,
        "ms_per_step": round(step_s * 1e3, 3), "scaling": "weak", "dtype": "u32 (SHA-256) + fp32",
        "data": "synthetic serialized updates (pickled {'w': 25M fp32}, device-PRNG payload) in pinned memory",
        "config": {"workload": f"cfg5 at arrival: {K} messages x {nbytes:,} B landed from the inbox's pinned "
                               f"buffers with host SHA-256 beside the DMAs, {len(bad)} corrupted, drop-in FedAvg "
                               f"over the {K - len(bad)} accepted", "parallelism": "single GPU, host hashing"},
        "roofline": {"bound": "host SHA-NI threads / PCIe H2D", "achieved": round(hashed / step_s / 1e9, 2),
                     "peak": round(bound, 2), "unit": "GB/s", "frac": round(hashed / step_s / 1e9 / bound, 4),
                     "traffic": None, "host_sha_bound_gbs": round(sha_gbs, 2), "pcie_h2d_gbs": round(h2d_gbs, 2),
                     "peak_what": "min(the product's hashing pool over these K pinned messages with nothing beside "
                                  "it; pinned H2D over PCIe), both measured on this box in this run"},
        "cpu_baseline": cpu}


# ------------------------------------------------------------------ delta / inbox
def run_delta_workload(args, n, seed, dev):
    """Trainer-side local update (reference node/node.py:273-282) of one
    flat n-parameter model: delta = cur - prev; prev = cur.  One GPU."""
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
        ok = bits_equal(delta[:m].cpu().numpy(), want) and torch.equal(prev[:m], cur[:m])
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
    ref_s = None
    if not args.no_reference_gpu:  # the reference's ops on this GPU: a sub and a clone (node.py:279,282)
        for i in range(3):
            if i == 1:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            d, c = cur - prev, cur.clone()
        torch.cuda.synchronize()
        ref_s = (time.perf_counter() - t0) / 2
        del d, c
    cpu = None
    if not args.no_cpu_baseline:
        import oracle.cpu_baseline as cb  # baseline leg only

        n_s = 50_000_000
        res = cb.delta(n_s, args.cpu_seconds)
        cpu = cpu_record(res, "GB/s", "port", f"{n_s:,} fp32 params, reference ops cur - prev and clone "
                                              f"(node/node.py:279,282) on torch CPU, {res['reps']} reps")
    del cur, prev, delta
    torch.cuda.empty_cache()
    return {
        "workload": "delta", "value": round(alg / step_s / 1e9, 2), "unit": "GB/s", "steps": args.steps,
        "ms_per_step": round(step_s * 1e3, 4), "scaling": "weak", "dtype": "fp32",
        "data": "synthetic (device counter PRNG); value = algorithmic bytes (16 B/param) per second",
        "config": {"workload": f"delta: trainer local update over {n:,} fp32 params (SURVEY §8(f) row 2)",
                   "coords_per_gpu": n, "parallelism": "single GPU (replicas only)"}
                  | ({"reference_on_gpu_ms_per_step": round(ref_s * 1e3, 3),
                      "speedup_vs_reference_on_gpu": round(ref_s / step_s, 2)} if ref_s else {}),
        "roofline": dict(roofline(alg, kern_ms, None), traffic=traffic_for("delta", n, 1)),
        "cpu_baseline": cpu}


def run_inbox_workload(args, K, n, seed, dev):
    """Receive path (reference node/node.py:135-138): K serialized updates of
    a GPU sender (pickle of CUDA tensors, node/node.py:285) deserialized into
    device tensors -- the reference's pickle.loads vs DeviceInbox.land.
    value = update bytes landed per second (host-to-device, PCIe-bound)."""
    import hashlib
    import pickle

    from p2pdl_amd.node.inbox import DeviceInbox

    shapes = resnet18_param_shapes()
    keys = [nm for nm, _ in shapes]
    ser = []
    for p in range(K):
        upd = {}
        for i, (k, s) in enumerate(shapes):
            t = torch.empty(s, dtype=torch.float32, device=dev)
            ops.fill_synthetic_(t.view(-1), seed, p * 1000 + i, UPD_SCALE)
            upd[k] = t
        ser.append(pickle.dumps(upd))  # what a CUDA trainer sends
    template = {k: torch.empty(s, dtype=torch.float32, device=dev) for k, s in shapes}
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

    # + the tester's per-update digest (its echo signs the serialized update,
    # node/node.py:144 -> utils/crypto.py:54-57): overlapped in land() vs after it
    def ours_digest():
        inbox.reset()
        for s in ser:
            inbox.land(s, digest=True)
        return [inbox.digest(k) for k in range(len(ser))]

    def land_then_hash():
        inbox.reset()
        for s in ser:
            inbox.land(s)
            hashlib.sha256(s).digest()

    def reference_echo():
        for s in ser:
            pickle.loads(s)
            hashlib.sha256(s).digest()

    if not args.no_check:
        ok = ours_digest() == [hashlib.sha256(s).digest() for s in ser]
        log(f"overlapped digests == hashlib: {ok}")
        if not ok:
            raise SystemExit("bench: inbox digest differs from hashlib")
    # the product receive path: DeviceInbox.recv puts each message in a pinned
    # buffer of the inbox (socket recv_into -- here a copy OUTSIDE the timed
    # region), and land() moves it in one DMA + the landing kernel
    msgs = [inbox.message_buffer(len(s)) for s in ser]
    for m, s in zip(msgs, ser):
        m.buf[:len(s)].copy_(torch.frombuffer(bytearray(s), dtype=torch.uint8))
    if not args.no_check:
        inbox.reset()
        got = inbox.land(msgs[0], 0)
        ref = pickle.loads(ser[0])
        torch.cuda.synchronize()
        ok = all(torch.equal(got[k], ref[k]) for k in keys)
        log(f"pinned landing (p2p_land_segments_f32) == pickle.loads: {ok}")
        if not ok:
            raise SystemExit("bench: pinned landing differs from pickle.loads")

    def ours_pinned():
        inbox.reset()
        for m in msgs:
            inbox.land(m)

    def ours_pinned_digest():
        inbox.reset()
        for m in msgs:
            inbox.land(m, digest=True)
        return [inbox.digest(k) for k in range(len(msgs))]

    t_pin, t_pin_dig = timed(ours_pinned), timed(ours_pinned_digest)
    t_ours, t_ref = timed(ours), timed(reference)
    t_dig, t_seq, t_ref_dig = timed(ours_digest), timed(land_then_hash), timed(reference_echo)
    n = sum(_numel(s) for _, s in shapes)
    nbytes = K * n * 4
    del inbox, template, msgs
    torch.cuda.empty_cache()
    return {
        "workload": "inbox", "value": round(nbytes / t_pin / 1e9, 3), "unit": "GB/s", "steps": args.steps,
        "ms_per_step": round(t_pin * 1e3, 3), "scaling": "weak",
        "dtype": "fp32", "data": "synthetic ResNet-18 updates pickled from CUDA tensors",
        "config": {"workload": f"inbox: land {K} serialized updates of {n:,} params ({len(shapes)} tensors) "
                               f"in the device slab (SURVEY §8(f) row 1)", "reference_pickle_loads_gbs":
                   round(nbytes / t_ref / 1e9, 3), "reference_ms": round(t_ref * 1e3, 3),
                   "timing": "value = messages in the inbox's pinned receive buffers (DeviceInbox.recv): one "
                             "DMA per message + the landing kernel; staging_* = bytes in pageable memory: memcpy "
                             "into a pinned staging row + one DMA",
                   "staging_ms": round(t_ours * 1e3, 3), "staging_gbs": round(nbytes / t_ours / 1e9, 3),
                   "pinned_digest_overlapped_ms": round(t_pin_dig * 1e3, 3),
                   "with_digest": {"land_digest_overlapped_ms": round(t_dig * 1e3, 3),
                                   "land_then_hashlib_ms": round(t_seq * 1e3, 3),
                                   "reference_pickle_loads_then_hashlib_ms": round(t_ref_dig * 1e3, 3),
                                   "what": "SHA-256 of each serialized update (the bytes the tester's echo "
                                           "signs) on a hashing thread beside parse + copy + DMA"},
                   "parallelism": "single GPU, host-to-device"},
        "roofline": {"bound": "pcie (host-to-device)", "achieved": round(nbytes / t_pin / 1e9, 2), "peak": 63.0,
                     "unit": "GB/s", "frac": round(nbytes / t_pin / 1e9 / 63.0, 4), "traffic": None},
        "cpu_baseline": {"value": round(nbytes / t_ref / 1e9, 3), "unit": "GB/s", "kind": "reference",
                         "cores": 1, "sample": f"the reference's own pickle.loads of the same {K} messages "
                                               f"(node/node.py:135), same process"}}


def run_digest_flow(args, steps):
    """The reference's per-round digest work, through the
    product's sign_data / verify_signature with the reference's call
    signatures: 3 trainers' serialized MNIST-MLP updates (node/node.py:285),
    4 testers -- 12 echo signs over each tester's own copy (node/node.py:145
    -> utils/broadcast.py:14), 12 echo verifies over the trainer's
    local_update (:155), 48 ready verifies over each ready message's copy
    (:175,:202): 72 SHA-256 passes in the reference (ECDSA(SHA256()) hashes
    its input on every call).  The objects are the ones the reference
    holds: each copy comes out of its own pickle round trip.  The EC step is
    stubbed on both sides (`cryptography` is absent from the image; it costs
    the same per signature either way).  Each step is a new round: the
    digest cache starts empty."""
    import hashlib
    import pickle

    import numpy as np

    from p2pdl_amd.utils import crypto, digests

    class Key:  # ECDSA stand-in over the 32-byte digest
        def sign(self, digest, alg):
            return b"sig:" + digest

        def verify(self, signature, digest, alg):
            if signature != b"sig:" + digest:
                raise ValueError("bad signature")

    fake = (types.SimpleNamespace(SHA256=lambda: None), types.SimpleNamespace(ECDSA=lambda a: a),
            types.SimpleNamespace(Prehashed=lambda h: h))
    saved_ec = crypto._ec
    crypto._ec = lambda: fake
    ks, key = crypto.KeyServer(), Key()
    ks.register_key("127.0.0.1", 1, key)
    testers = 4
    try:
        def make_round(seed):
            ups = []
            for t in range(3):
                rng = np.random.default_rng(seed * 10 + t)
                ups.append(pickle.dumps({nm: torch.from_numpy(rng.standard_normal(s, dtype=np.float32) * 1e-2)
                                         for nm, s in MLP_SHAPES}))
            copies = [[pickle.loads(pickle.dumps({"model": u}))["model"] for u in ups] for _ in range(testers)]
            ready = [[pickle.loads(pickle.dumps({"local_update": u}))["local_update"] for u in ups]
                     for _ in range(testers)]
            return ups, copies, ready

        def product(ups, copies, ready):
            sig = {}
            for i in range(testers):
                for t in range(3):
                    sig[i, t] = crypto.sign_data(key, copies[i][t])
            ok = 0
            for t in range(3):
                for i in range(testers):
                    ok += crypto.verify_signature(ks, "127.0.0.1", 1, ups[t], sig[i, t])
            for i in range(testers):
                for t in range(3):
                    for j in range(testers):
                        ok += crypto.verify_signature(ks, "127.0.0.1", 1, ready[i][t], sig[j, t])
            return sig, ok

        def reference(ups, copies, ready):
            out = []
            for i in range(testers):
                for t in range(3):
                    out.append(hashlib.sha256(copies[i][t]).digest())
            for t in range(3):
                for i in range(testers):
                    out.append(hashlib.sha256(ups[t]).digest())
            for i in range(testers):
                for t in range(3):
                    for j in range(testers):
                        out.append(hashlib.sha256(ready[i][t]).digest())
            return out

        t_prod, t_ref, misses = [], [], []
        for step in range(steps + 1):
            rnd = make_round(step)
            digests.CACHE.clear()
            m0 = digests.CACHE.misses
            t0 = time.perf_counter()
            sig, ok = product(*rnd)
            t1 = time.perf_counter()
            ref = reference(*rnd)
            t2 = time.perf_counter()
            if ok != 60 or any(sig[i, t] != b"sig:" + hashlib.sha256(rnd[0][t]).digest()
                               for i in range(testers) for t in range(3)):
                raise SystemExit("bench: digest_flow signatures differ from hashlib")
            if step:  # step 0 warms up
                t_prod.append(t1 - t0)
                t_ref.append(t2 - t1)
                misses.append(digests.CACHE.misses - m0)
        msg = len(rnd[0][0])
    finally:
        crypto._ec = saved_ec
        digests.CACHE.clear()
    tp, tr = min(t_prod), min(t_ref)
    log(f"digest_flow: product {tp*1e3:.3f} ms ({misses[-1]} hashes) vs reference {tr*1e3:.3f} ms (72 hashes)")
    hashed = 72 * msg
    return {
        "workload": "digest_flow", "value": round(hashed / tp / 1e9, 3), "unit": "GB/s", "steps": steps,
        "ms_per_step": round(tp * 1e3, 4), "scaling": "weak", "dtype": "u32 (SHA-256)",
        "data": "synthetic MNIST-MLP updates (models/model.py:6-8) pickled like node/node.py:285",
        "config": {"workload": f"digest_flow: one round's 72 sign/verify digests over 3 updates of {msg:,} B, "
                               f"4 testers (SURVEY.md §3D), reference call signatures, best of {steps} rounds",
                   "reference_ms": round(tr * 1e3, 4), "speedup_vs_reference": round(tr / tp, 2),
                   "hashes_product": misses[-1], "hashes_reference": 72, "message_bytes": msg,
                   "parallelism": "host (one process)"},
        "roofline": None,
        "cpu_baseline": {"value": round(hashed / tr / 1e9, 3), "unit": "GB/s", "kind": "reference", "cores": 1,
                         "sample": "the reference's 72 hashlib.sha256 passes (ECDSA(SHA256()) at "
                                   "utils/crypto.py:56,95) over the same objects, same process"}}


def run_broadcast_workload(args, seed, dev):
    """Global-model serialization before the broadcast (SURVEY §8(f) row 4;
    reference aggregator/aggregation.py:66-70): the tester pickles its
    ResNet-18-sized state_dict into the 'global_model_update' envelope.  The
    reference pickles the CUDA state_dict: torch copies every tensor to the
    host, into a BytesIO, out of it and into the pickle.  The product
    (node/envelope.py) DMAs each fp32 tensor into a pinned slot laid out as
    torch's storage blob and pickles the slots in-band (protocol 5): the
    joined envelope costs one copy of the weights; the parts the broadcast
    sends (envelope_parts) none.  value = model bytes serialized per second
    into the parts the broadcast sends (device-to-host + pickle);
    joined_ms: the same into one bytes object."""
    import pickle

    from p2pdl_amd.node import envelope as env

    shapes = resnet18_param_shapes()
    model = torch.nn.Module()
    for i, (nm, shape) in enumerate(shapes):
        t = torch.empty(shape, dtype=torch.float32, device=dev)
        ops.fill_synthetic_(t.view(-1), seed, i, W_SCALE)
        model.register_parameter(nm.replace(".", "__"), torch.nn.Parameter(t, requires_grad=False))
    torch.cuda.synchronize()

    def envelope(state):
        return pickle.dumps({"type": "global_model_update", "model": state, "addr": "127.0.0.1", "port": 1})

    def ours():
        return env.global_model_envelope(model.state_dict(), "127.0.0.1", 1)

    def ours_parts():
        with env.LOCK:
            return sum(p.nbytes for p in env.envelope_parts(model.state_dict(), "127.0.0.1", 1))

    def reference():
        return envelope(model.state_dict())

    if not args.no_check:
        a, b = pickle.loads(ours())["model"], pickle.loads(reference())["model"]
        ok = list(a) == list(b) and all(a[k].device == b[k].device and torch.equal(a[k], b[k]) for k in b)
        log(f"broadcast: envelope == the reference's (payloads, devices): {ok}")
        if not ok:
            raise SystemExit("bench: broadcast payload differs from the reference's")

    def timed(fn):
        for _ in range(max(args.warmup, 1)):
            fn()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        return (time.perf_counter() - t0) / args.steps

    # the broadcast's own path: the parts it sends (node.envelope.envelope_parts);
    # the joined bytes object beside it
    t_joined, t_ref, t_ours = timed(ours), timed(reference), timed(ours_parts)
    nbytes = 4 * sum(_numel(s) for _, s in shapes)
    del model
    torch.cuda.empty_cache()
    return {
        "workload": "broadcast", "value": round(nbytes / t_ours / 1e9, 3), "unit": "GB/s", "steps": args.steps,
        "ms_per_step": round(t_ours * 1e3, 3), "scaling": "weak", "dtype": "fp32",
        "data": "synthetic ResNet-18-sized model on the GPU",
        "config": {"workload": f"broadcast: the global_model_update envelope of a {len(shapes)}-tensor state_dict "
                               f"({nbytes / 4:,.0f} params) pickled from the GPU model (SURVEY §8(f) row 4)",
                   "reference_ms": round(t_ref * 1e3, 3), "speedup_vs_reference": round(t_ref / t_ours, 2),
                   "joined_ms": round(t_joined * 1e3, 3),
                   "speedup_joined_vs_reference": round(t_ref / t_joined, 2),
                   "parallelism": "single GPU, device-to-host"},
        "roofline": {"bound": "pcie (device-to-host) + host pickle", "achieved": round(nbytes / t_ours / 1e9, 2),
                     "peak": 63.0, "unit": "GB/s", "frac": round(nbytes / t_ours / 1e9 / 63.0, 4), "traffic": None},
        "cpu_baseline": {"value": round(nbytes / t_ref / 1e9, 3), "unit": "GB/s", "kind": "reference", "cores": 1,
                         "sample": "the reference's pickle.dumps of the CUDA state_dict envelope "
                                   "(aggregation.py:70), same process"}}


def replica_workload(args, name, dev):
    """cfg5 / sha256 / delta / inbox / broadcast (one GPU each): the workload's record."""
    rule, K, n, seed = WORKLOADS[name]
    if name == args.workload:
        K, n = args.peers or K, args.coords or n
    if rule in ("fused", "sha256"):
        return run_digest_workload(args, rule, K, n, seed, dev)
    if rule == "digest-flow":
        return run_digest_flow(args, args.steps)
    if rule == "delta":
        return run_delta_workload(args, n, seed, dev)
    if rule == "broadcast":
        return run_broadcast_workload(args, seed, dev)
    if rule == "arrival":
        return run_cfg5_arrival(args, K, n, seed, dev)
    return run_inbox_workload(args, K, n, seed, dev)


# ------------------------------------------------------------------ main
SUB_KEEP = ("us_per_call", "us_per_call_general_path", "ms_per_job", "kernel_ms_sum", "allgather_ms_sum")
ROOF_KEEP = ("bound", "kernel_ms", "call_ms", "vs_flat_kernel", "digest_route", "digest_ms", "host_sha_bound_gbs",
             "pcie_d2h_gbs", "pcie_h2d_gbs", "fedavg_kernel_ms", "fedavg_frac_of_hbm_peak", "sha256_kernel_gbs")
CFG_KEEP = ("per_rank", "world_size", "rccl_version")


def compact_sub(rec: dict) -> dict:
    """A sub-record as printed on the driver's line: the numbers only (the
    workload definitions are WORKLOADS / the docstring above), so the whole
    line -- cfg3_full included -- fits the driver's stdout tail."""
    out = {"value": rec["value"], "unit": rec["unit"]}
    if "ms_per_step" in rec:
        out["ms"] = rec["ms_per_step"]
    out.update({k: rec[k] for k in SUB_KEEP if k in rec})
    if rec.get("general_path"):
        out["general_path"] = {a: b for a, b in rec["general_path"].items() if a != "what"}
    if rec.get("reference_on_gpu"):
        out["reference_on_gpu"] = {a: b for a, b in rec["reference_on_gpu"].items() if a != "what"}
    roof = rec.get("roofline") or {}
    if roof:
        out["frac"] = roof.get("frac")
        out.update({k: roof[k] for k in ROOF_KEEP if k in roof})
        alg, tr = roof.get("alg_bytes_per_launch"), roof.get("traffic")
        if alg and tr:
            out["traffic_x"] = round(tr / alg, 5)
    cfg = rec.get("config") or {}
    out.update({k: cfg[k] for k in CFG_KEEP if k in cfg})
    for k in ("reference_ms", "staging_ms", "pinned_digest_overlapped_ms", "with_digest", "hashes_product",
              "speedup_vs_reference", "joined_ms", "reference_on_gpu_ms_per_step", "speedup_vs_reference_on_gpu"):
        if k in cfg:
            v = cfg[k]
            out[k] = {a: b for a, b in v.items() if a != "what"} if isinstance(v, dict) else v
    cpu = rec.get("cpu_baseline")
    if cpu:
        out["cpu"] = {k: cpu[k] for k in ("value", "unit", "cores", "value_1thread", "us_per_call", "kind")
                      if k in cpu}
    return out


HBM_BYTES = 288e9
XGMI_LINK_GBS = 153.0  # one xGMI link (7 per GPU): a single ring's per-link bound


def scale_plan(world: int, n1: dict, *, steps: int = 10, warmup: int = 2, chunks: int = 8,
               fill_tbs: float = 1.0, startup_s: float = 120.0) -> dict:
    """The default line's footprint and run time at ``world`` GPUs, predicted
    from the measured N = 1 line ``n1`` (its ms_per_step and sub.cfg3_full
    ms_per_job) -- no GPU needed.  Per rank: the main line's resident [K, n]
    slab + w + the all-gathered model, then cfg3_full's 125M-coordinate tile
    + the 1B-coordinate model; time: the inputs generated on device (at
    ``fill_tbs``), warmup + timed steps, cfg3_full's 8 / world tiles per pass
    (two passes), each chunk's all-gather bounded by one ring per link, and a
    fixed allowance for the first torch import and RCCL's setup."""
    K, n = 256, CFG3_TILE
    main_bytes = (K + 2 + world) * n * 4 if world > 1 else (K + 2) * n * 4
    full_bytes = K * CFG3_TILE * 4 + CFG3_TILE * 4 + (CFG3_COORDS * 4 if world > 1 else 0)
    step_ms = float(n1["ms_per_step"])
    C = n // chunks
    gather_ms = 0.0 if world == 1 else chunks * C * 4 * (world - 1) / (XGMI_LINK_GBS * 1e9) * 1e3
    step_pred = max(step_ms, gather_ms) + (gather_ms / chunks if world > 1 else 0.0)  # the last chunk's gather
    tiles = CFG3_COORDS // CFG3_TILE // world
    job_ms = float(n1["sub"]["cfg3_full"]["ms_per_job"]) * tiles / (CFG3_COORDS // CFG3_TILE) if n1.get("sub") else \
        step_ms * tiles
    fill_s = (K + 1) * n * 4 / (fill_tbs * 1e12)
    total_s = startup_s + fill_s + (steps + warmup) * step_pred / 1e3 + 2 * tiles * (fill_s + job_ms / 1e3)
    if world > 1:  # the other exchange legs (config.gather_legs), 1 + min(steps, 5) steps each, priced in line
        total_s += (len(GATHER_LEGS) - 1) * (fill_s + (1 + min(steps, 5)) * (step_ms + gather_ms) / 1e3)
    return {"world": world, "bytes_per_rank": max(main_bytes, full_bytes), "fits_hbm": max(main_bytes, full_bytes)
            < 0.97 * HBM_BYTES, "step_ms": round(step_pred, 3), "allgather_ms_per_step": round(gather_ms, 3),
            "seconds": round(total_s, 1)}


def launch_plan(gpus: int, env, visible: int, backend: str):
    """How this process runs ``--gpus N`` (no GPU is touched here):
      ("spawn", N)  WORLD_SIZE unset and N > 1: start N ranks as children
                    (torch.distributed.run, one process per GPU) and relay;
      ("rank", W)   inside a launcher (WORLD_SIZE = W) or N == 1: run as a rank.
    A launcher world that differs from --gpus, or an RCCL world larger than
    the visible GPUs, is an error (SystemExit), never a silent 1-GPU line."""
    if gpus < 1:
        raise SystemExit(f"bench: --gpus must be >= 1, got {gpus}")
    ws = env.get("WORLD_SIZE")
    if ws is None:
        world = gpus
        if gpus == 1:
            return "rank", 1
    else:
        world = int(ws)
        if world != gpus:
            raise SystemExit(f"bench: WORLD_SIZE={world} from the launcher but --gpus {gpus}")
    if world > 1 and backend == "nccl" and visible < world:
        raise SystemExit(f"bench: --gpus {world} over RCCL needs {world} GPUs, {visible} visible "
                         f"(P2P_DIST_BACKEND=gloo rehearses several ranks on one GPU)")
    return ("spawn", world) if ws is None else ("rank", world)


def spawn_command(gpus: int, port: int, argv) -> list:
    """The child launch of ``--gpus N`` without an outer launcher: one rank per
    GPU on this node, rendezvous on 127.0.0.1 (the driver's own N > 1 form)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


@contextlib.contextmanager
def stdout_to_stderr():
    """File descriptor 1 points at stderr inside the block (native libraries
    printing to stdout included); Python's own stdout is flushed first."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        os.dup2(saved, 1)
        os.close(saved)


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    args = parse()
    # P2P_DIST_BACKEND=gloo rehearses N>1 on a single GPU (ranks share cuda:0);
    # the driver's multi-GPU runs use nccl (= RCCL over xGMI), one GPU per rank.
    backend = os.environ.get("P2P_DIST_BACKEND", "nccl")
    visible = torch.cuda.device_count()  # does not initialise the GPU on this image
    mode, world = launch_plan(args.gpus, os.environ, visible, backend)
    if mode == "spawn":
        # this parent never touches the GPU: the ranks are its children and
        # rank 0's JSON line reaches our stdout directly
        import subprocess

        cmd = spawn_command(world, _free_port(), sys.argv[1:])
        log(f"bench: --gpus {world}: launching {world} ranks ({backend}): {' '.join(cmd)}")
        sys.exit(subprocess.call(cmd))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % max(1, visible)
    if world > 1:
        import datetime

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        # a collective stuck longer than this ends the rank non-zero with the
        # collective named (the process group's watchdog), well inside the
        # driver's run limit, instead of a silent hang
        tmo = datetime.timedelta(seconds=float(os.environ.get("P2P_DIST_TIMEOUT_S", "240")))
        # stdout carries one JSON line: what the backends print while they
        # connect (gloo's "[Gloo] Rank r is connected to ...", RCCL's
        # NCCL_DEBUG lines) goes to stderr
        with stdout_to_stderr():
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
            else:
                dist.init_process_group(backend, timeout=tmo)
            dist.barrier()
        if dist.get_world_size() != world:
            raise SystemExit(f"bench: process group has {dist.get_world_size()} ranks, expected {world}")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    c = Ctx(world=world, rank=rank, dev=dev, backend=backend)

    rule, K, n, seed = WORKLOADS[args.workload]
    K = args.peers or K
    n = args.coords or n
    one_gpu = {"fused": "cfg5/sha256 run as replicas only", "sha256": "cfg5/sha256 run as replicas only",
               "digest-flow": "digest-flow runs in one process", "broadcast": "broadcast runs on one GPU",
               "arrival": "cfg5-arrival runs as replicas only",
               "delta": "delta runs as replicas only", "inbox": "inbox runs on one GPU", "dropin": "drop-in runs on one GPU"}
    if rule in one_gpu and world > 1:
        raise SystemExit(one_gpu[rule] + " (one process per GPU)")
    if rule in ("fused", "sha256", "delta", "inbox", "digest-flow", "broadcast", "arrival"):
        rec = replica_workload(args, args.workload, dev)
        print(json.dumps({"metric": METRIC, "value": rec["value"], "unit": rec["unit"], "n_gpus": 1,
                          "steps": rec["steps"], "warmup": args.warmup, "ms_per_step": rec["ms_per_step"],
                          "higher_is_better": True, "scaling": rec["scaling"], "vs_baseline": None,
                          "dtype": rec["dtype"], "data": rec["data"], "config": rec["config"],
                          "roofline": rec["roofline"], "cpu_baseline": rec["cpu_baseline"]}), flush=True)
        return

    data = "synthetic (device counter PRNG, SURVEY.md §8(d)); random-init model weights"
    if args.job == "cfg3-full":
        rec = measure_cfg3_full(c, args, passes=max(1, args.steps), gather=args.gather)
        main_rec, steps, step_ms = rec, 1, rec["ms_per_job"]
        sub = {}
    else:
        if rule == "dropin":
            main_rec = measure_dropin(c, args, args.workload, K, seed, max(args.steps, 20), args.warmup,
                                      args.cpu_seconds)
            step_ms = main_rec["ms_per_step"]
        else:
            main_rec, step_s = measure_flat(c, args, args.workload, rule, K, n, seed, args.steps, args.warmup,
                                            args.cpu_seconds, args.chunks, gather=args.gather)
            step_ms = step_s * 1e3
            if world > 1 and not args.no_sub:
                # the other exchange legs, same data and plan, fewer steps:
                # one driver run carries all three (VERDICT r05 next #4 and
                # weak #7: in line, overlapped, and the direct exchange)
                legs = {args.gather: {"ms_per_step": round(step_ms, 4), "value": main_rec["value"],
                                      "pipeline": main_rec["config"].get("pipeline")}}
                for other in GATHER_LEGS:
                    if other == args.gather:
                        continue
                    try:
                        o_rec, o_s = measure_flat(c, args, args.workload, rule, K, n, seed, min(args.steps, 5), 1,
                                                  0, args.chunks, gather=other)
                    except (RuntimeError, dist.DistBackendError) as e:  # a leg's failure is its record, not the line's
                        legs[other] = {"error": f"{type(e).__name__}: {e}"[:300]}
                        torch.cuda.synchronize()
                        continue
                    legs[other] = {"ms_per_step": o_rec["ms_per_step"], "value": o_rec["value"],
                                   "pipeline": o_rec["config"].get("pipeline"),
                                   "per_rank": o_rec["config"].get("per_rank")}
                main_rec["config"]["gather_legs"] = legs
        steps = main_rec["steps"]
        sub = {}
        if not args.no_sub and args.workload == "cfg3" and not (args.coords or args.peers):
            sub["cfg3_full"] = measure_cfg3_full(c, args, gather=args.gather)
            if main_rec.get("cpu_baseline"):  # the same rule and op sequence as the main line
                sub["cfg3_full"]["cpu_baseline"] = dict(main_rec["cpu_baseline"], note="the cfg3 line's CPU run "
                                                        "(same rule, per-coordinate cost independent of N)")
            if world == 1:
                for name in SUB_N1:
                    r, k2, n2, s2 = WORKLOADS[name]
                    if r == "dropin":
                        rec = measure_dropin(c, args, name, k2, s2, 30, 2, args.sub_cpu_seconds)
                    elif r in ("fused", "delta", "inbox", "digest-flow", "broadcast", "arrival"):
                        sargs = argparse.Namespace(**dict(vars(args), workload=name, steps=SUB_STEPS[name],
                                                          warmup=1, cpu_seconds=args.sub_cpu_seconds))
                        rec = replica_workload(sargs, name, dev)
                        rec["workload"] = name
                    else:
                        rec, _ = measure_flat(c, args, name, r, k2, n2, s2, 10, 2, args.sub_cpu_seconds, 1)
                    sub[rec["workload"]] = rec
    if rank == 0:
        line = {
            "metric": METRIC, "value": main_rec["value"], "unit": "GB/s", "n_gpus": world, "steps": steps,
            "warmup": args.warmup, "ms_per_step": round(step_ms, 4), "higher_is_better": True,
            "scaling": main_rec["scaling"], "vs_baseline": None, "dtype": main_rec["dtype"], "data": data,
            "config": main_rec["config"], "roofline": main_rec["roofline"],
            "cpu_baseline": main_rec.get("cpu_baseline"),
        }
        if main_rec.get("general_path"):
            line["general_path"] = main_rec["general_path"]
        if sub:
            line["sub"] = {k: compact_sub(v) for k, v in sub.items()}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
