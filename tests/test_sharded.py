"""Coordinate sharding + all-gather over gloo, world size 2, on CPU.

The per-shard reduce is the CPU oracle injected through sharded_aggregate_'s
``reduce`` seam (test-only); what is under test is the plan, the ragged tail,
and that the gathered model is byte-identical to the unsharded result.  The
GPU leg (same code with the HIP reduce and RCCL) runs in bench.py at N > 1.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from p2pdl_amd import sharded
from p2pdl_amd.sharded import ChunkPlan, sharded_aggregate_


def test_chunk_plan_covers_every_coordinate_once():
    for n, world, chunk in [(1000, 2, 64), (1000, 3, 7), (5, 4, 16), (4096, 8, 512), (1, 2, 1)]:
        seen = np.zeros(n, dtype=int)
        for r in range(world):
            plan = ChunkPlan(n, world, chunk)
            for st, ln in plan.owned(r):
                seen[st:st + ln] += 1
            assert plan.local_len(r) == sum(ln for _, ln in plan.owned(r))
        assert (seen == 1).all(), (n, world, chunk)


@pytest.mark.parametrize("k,n,at_least,want", [
    (256, 125_000_000, 1, 8),    # cfg3 tile: 128 GB -> 8 planes of 16 GB
    (256, 125_000_000, 8, 8),    # N > 1: the all-gather chunks already fit
    (256, 100_000_000, 1, 8),    # 102 GB: 7 would do, 8 divides 100M
    (128, 100_000_000, 1, 4),    # cfg4: 51 GB
    (64, 11_689_512, 1, 1),      # cfg2: 3 GB, one plane
    (256, 7, 1, 1),
    (4, 13, 2, 13),              # nothing between 2 and 13 divides a prime
])
def test_plane_count(k, n, at_least, want):
    s = sharded.plane_count(k, n, at_least)
    assert s == want and n % s == 0
    assert s == 1 or k * (n // s) * 4 <= sharded.PLANE_BYTES or s == n


def test_plane_count_refuses_an_unsplittable_size():
    with pytest.raises(ValueError, match="divides"):
        sharded.plane_count(256, 1_000_000_007)  # prime, 128 GB: no even split near 8 planes


@pytest.mark.gpu
def test_peer_planes_layout_and_reduce(cuda):
    """PeerPlanes: chunk-major planes, 256-B aligned rows, one table per
    plane; reduce_ over each plane equals one flat reduction of the peers'
    concatenated chunks (bit-exact against the oracle)."""
    from p2pdl_amd import ops

    k, chunks, chunk, seed = 20, 3, 70_001, 0x91A
    planes = sharded.PeerPlanes(k, chunks, chunk, cuda)
    assert planes.data.shape == (chunks, k, 70_016) and planes.pitch % 64 == 0
    assert all(planes.row(s, p).data_ptr() % 256 == 0 for s in range(chunks) for p in range(k))
    assert planes.row(1, 0).data_ptr() - planes.row(0, k - 1).data_ptr() == planes.pitch * 4  # plane-major
    peers = [oracle.synth(chunks * chunk, seed, p, 1e-2) for p in range(k)]
    w = oracle.synth(chunks * chunk, seed, 0xFFFFF, 5e-2)
    for s in range(chunks):
        for p in range(k):
            planes.row(s, p).copy_(torch.from_numpy(peers[p][s * chunk:(s + 1) * chunk]))
    wt = torch.from_numpy(w.copy()).to(cuda)
    for s in range(chunks):
        planes.reduce_(s, wt[s * chunk:(s + 1) * chunk], "fedavg")
    w_ref, _ = oracle.fedavg(peers, w)
    assert np.array_equal(wt.cpu().numpy().view(np.uint32), w_ref.view(np.uint32))
    with pytest.raises(ValueError):  # a w longer than the plane's rows
        planes.reduce_(0, torch.zeros(chunk + 1, device=cuda))


@pytest.mark.gpu
def test_peer_planes_whole_rounds_on_the_split_kernel(cuda):
    """round_plane_sizes' layout through the HIP path: planes of whole CU
    rounds (the split kernel alone) and a short last plane (split rounds + the
    VGPR remainder), one aggregate_gather_ into w_full, bit-exact against the
    oracle; K = 16, the split kernel's smallest K."""
    k, seed = 16, 0x91B
    R = torch.cuda.get_device_properties(cuda).multi_processor_count * 8192
    sizes = [2 * R, 2 * R, R + 3 * 8192 + 1000]
    n = sum(sizes)
    planes = sharded.PeerPlanes(k, 0, 0, cuda, sizes=sizes)
    peers = [oracle.synth(n, seed, p, 1e-2) for p in range(k)]
    w = oracle.synth(n, seed, 0xFFFFF, 5e-2)
    ws = []
    for s, (o, c) in enumerate(zip(planes.offsets, planes.sizes)):
        for p in range(k):
            planes.row(s, p).copy_(torch.from_numpy(peers[p][o:o + c]))
        ws.append(torch.from_numpy(w[o:o + c].copy()).to(cuda))
    w_full = torch.empty(n, device=cuda)
    planes.aggregate_gather_(ws, w_full)
    w_ref, _ = oracle.fedavg(peers, w)
    assert np.array_equal(w_full.cpu().numpy().view(np.uint32), w_ref.view(np.uint32))


def test_global_index_matches_device_prng_mapping():
    """Memory-sharded layout: local i -> global index == oracle.synth's chunk map."""
    plan = ChunkPlan(8 * 4 * 100, 4, 100)
    for r in range(4):
        gi = [plan.global_index(r, i) for i in range(plan.local_len(r))]
        a = oracle.synth(plan.local_len(r), 5, 1, 1.0, 100, 4, r)
        b = oracle.synth(plan.n, 5, 1, 1.0)[gi]
        assert np.array_equal(a, b)


def oracle_reduce(peers, w, rule, lr, trim_frac):
    rid = {"fedavg": 0, "median": 1, "trimmed": 2}[rule]
    ps = [p.numpy() for p in peers]
    if rid == 0:
        new, _ = oracle.fedavg(ps, w.numpy(), lr=lr)
    else:
        new, _ = oracle.robust(ps, rid, oracle.trim_count(len(ps), trim_frac) if rid == 2 else 0,
                               w=w.numpy(), lr=lr)
    w.copy_(torch.from_numpy(new))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, k, rule, chunk, q, exchange="all_gather"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        peers = [torch.from_numpy(oracle.synth(n, 17, p, 1e-2)) for p in range(k)]
        w = torch.from_numpy(oracle.synth(n, 17, 0xFFFFF, 5e-2))
        sharded_aggregate_(w, peers, rule=rule, chunk=chunk, reduce=oracle_reduce, exchange=exchange)
        q.put((rank, w.numpy().tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,rule,n,k,chunk,exchange", [
    (2, "fedavg", 10_007, 5, 1000, "all_gather"), (2, "fedavg", 4096, 3, 512, "all_gather"),
    (2, "median", 3001, 7, 256, "all_gather"), (2, "trimmed", 777, 10, 100, "all_gather"),
    # the driver's 4-rank leg and an odd world, rehearsed on gloo
    (4, "fedavg", 10_007, 6, 300, "all_gather"), (3, "median", 2049, 9, 128, "all_gather"),
    # the direct exchange (sharded.exchange_): same bytes, same places
    (2, "fedavg", 10_007, 5, 1000, "p2p"), (3, "fedavg", 10_007, 6, 300, "p2p"), (4, "trimmed", 2049, 9, 128, "p2p")])
def test_gloo_world_byte_identical_to_single(world, rule, n, k, chunk, exchange):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, k, rule, chunk, q, exchange))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    peers = [oracle.synth(n, 17, p, 1e-2) for p in range(k)]
    w = oracle.synth(n, 17, 0xFFFFF, 5e-2)
    if rule == "fedavg":
        want, _ = oracle.fedavg(peers, w)
    else:
        rid = 1 if rule == "median" else 2
        want, _ = oracle.robust(peers, rid, oracle.trim_count(k) if rid == 2 else 0, w=w)
    assert all(got[r] == want.tobytes() for r in range(world))


def _planes_worker(rank, world, port, n, k, rule, S, q, exchange="all_gather"):
    """Memory-sharded inputs: this rank holds only its owned chunks of every
    peer, in PeerPlanes (CPU tensors here; the oracle reduces), and one
    aggregate_gather_ reassembles the global model."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        C = n // (world * S)
        plan = ChunkPlan(n, world, C)
        owned = plan.owned(rank)
        assert len(owned) == S and plan.tail == 0
        peers = [oracle.synth(n, 29, p, 1e-2) for p in range(k)]
        w = oracle.synth(n, 29, 0xFFFFF, 5e-2)
        planes = sharded.PeerPlanes(k, S, C, "cpu")
        for s, (st, ln) in enumerate(owned):
            for p in range(k):
                planes.row(s, p).copy_(torch.from_numpy(peers[p][st:st + ln]))
        ws = [torch.from_numpy(w[st:st + ln].copy()) for st, ln in owned]
        w_full = torch.zeros(n, dtype=torch.float32)

        def reduce(pl, s, wchunk, rule_, lr, trim_frac):
            oracle_reduce([pl.row(s, p) for p in range(pl.k)], wchunk, rule_, lr, trim_frac)

        seen = []
        planes.aggregate_gather_(ws, w_full, rule=rule, reduce=reduce, hook=lambda s, ph, st: seen.append((s, ph)),
                                 exchange=exchange)
        assert seen == [(s, ph) for s in range(S) for ph in ("reduce0", "reduce1", "gather0", "gather1")]
        q.put((rank, w_full.numpy().tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,rule,n,k,S,exchange", [
    (2, "fedavg", 2 * 3 * 1001, 5, 3, "all_gather"), (2, "trimmed", 2 * 2 * 640, 10, 2, "all_gather"),
    (2, "fedavg", 2 * 3 * 1001, 5, 3, "p2p"), (4, "fedavg", 4 * 2 * 500, 3, 2, "p2p")])
def test_gloo_peer_planes_round_byte_identical_to_single(world, rule, n, k, S, exchange):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_planes_worker, args=(r, world, port, n, k, rule, S, q, exchange))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    peers = [oracle.synth(n, 29, p, 1e-2) for p in range(k)]
    w = oracle.synth(n, 29, 0xFFFFF, 5e-2)
    if rule == "fedavg":
        want, _ = oracle.fedavg(peers, w)
    else:
        want, _ = oracle.robust(peers, 2, oracle.trim_count(k), w=w)
    assert all(got[r] == want.tobytes() for r in range(world))


def test_peer_planes_one_rank_fills_w_full():
    """No process group: each plane's chunk lands at w_full[s*C:(s+1)*C]."""
    k, S, C = 4, 3, 50
    peers = [oracle.synth(S * C, 31, p, 1e-2) for p in range(k)]
    w = oracle.synth(S * C, 31, 0xFFFFF, 5e-2)
    planes = sharded.PeerPlanes(k, S, C, "cpu")
    for s in range(S):
        for p in range(k):
            planes.row(s, p).copy_(torch.from_numpy(peers[p][s * C:(s + 1) * C]))
    ws = [torch.from_numpy(w[s * C:(s + 1) * C].copy()) for s in range(S)]
    w_full = torch.zeros(S * C)
    planes.aggregate_gather_(ws, w_full, reduce=lambda pl, s, wc, r, lr, tf: oracle_reduce(
        [pl.row(s, p) for p in range(pl.k)], wc, r, lr, tf))
    want, _ = oracle.fedavg(peers, w)
    assert w_full.numpy().tobytes() == want.tobytes()
    with pytest.raises(ValueError, match="w_full"):
        planes.aggregate_gather_(ws, torch.zeros(S * C - 1), reduce=lambda *a: None)


def test_round_plane_sizes():
    R = 256 * 8192
    # the cfg3 tile: 8 CU rounds fill one 16-GiB plane of 256 rows exactly
    assert sharded.round_plane_sizes(256, 125_000_000, R) == [8 * R] * 7 + [125_000_000 - 56 * R]
    assert sharded.round_plane_sizes(256, 16 * R, R) == [8 * R] * 2          # no remainder plane
    assert sharded.round_plane_sizes(64, 11_689_512, R) == [11_689_512]       # fits one plane
    assert sharded.round_plane_sizes(4096, 10 * R, R) == [R] * 10              # at least one round
    for k, n in ((256, 125_000_000), (128, 100_000_000), (16, 46_758_048)):
        sizes = sharded.round_plane_sizes(k, n, R)
        assert sum(sizes) == n and all(c % R == 0 for c in sizes[:-1])
        assert all(4 * k * c <= sharded.PLANE_BYTES for c in sizes)


@pytest.mark.parametrize("world", [1, 2])
def test_peer_planes_unequal_sizes(world):
    """Planes of unequal lengths (a short last plane): every plane's chunk
    lands at its offset in w_full, byte-identical to the whole reduction;
    at world 2 (gloo, in-process ranks) round s gathers G chunks of sizes[s]."""
    k, sizes = 4, [40, 40, 13]
    n = sum(sizes) * world
    if world == 1:
        results = [_unequal_planes_rank(0, 1, None, k, sizes, n)]
    else:
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_unequal_planes_rank, args=(r, world, port, k, sizes, n, q))
                 for r in range(world)]
        for p in procs:
            p.start()
        results = [q.get(timeout=120) for _ in procs]
        for p in procs:
            p.join(60)
            assert p.exitcode == 0
    peers = [oracle.synth(n, 37, p, 1e-2) for p in range(k)]
    w = oracle.synth(n, 37, 0xFFFFF, 5e-2)
    want, _ = oracle.fedavg(peers, w)
    assert all(r == want.tobytes() for r in results)


def _unequal_planes_rank(rank, world, port, k, sizes, n, q=None):
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        peers = [oracle.synth(n, 37, p, 1e-2) for p in range(k)]
        w = oracle.synth(n, 37, 0xFFFFF, 5e-2)
        planes = sharded.PeerPlanes(k, 0, 0, "cpu", sizes=sizes)
        assert planes.chunks == 3 and planes.chunk == 40 and planes.offsets == [0, 40, 80]
        ws = []
        for s, (o, c) in enumerate(zip(planes.offsets, planes.sizes)):
            st, ln = planes.global_range(s, rank, world)
            assert (st, ln) == (o * world + rank * c, c)  # round s: G chunks of sizes[s], rank order
            assert planes.global_index(s, rank, world, c - 1) == st + c - 1
            for p in range(k):
                planes.row(s, p).copy_(torch.from_numpy(peers[p][st:st + c]))
            ws.append(torch.from_numpy(w[st:st + c].copy()))
        w_full = torch.zeros(n)
        planes.aggregate_gather_(ws, w_full, reduce=lambda pl, s, wc, r, lr, tf: oracle_reduce(
            [pl.row(s, p) for p in range(pl.k)], wc, r, lr, tf))
        out = w_full.numpy().tobytes()
        if q is not None:
            q.put(out)
        return out
    finally:
        if world > 1:
            dist.destroy_process_group()


def test_exchange_refuses_an_unknown_kind():
    planes = sharded.PeerPlanes(2, 1, 10, "cpu")
    with pytest.raises(ValueError, match="exchange"):
        planes.aggregate_gather_([torch.zeros(10)], reduce=lambda *a: None, exchange="ring")
    with pytest.raises(ValueError, match="exchange"):
        sharded_aggregate_(torch.zeros(10), [torch.zeros(10)], reduce=lambda *a: None, exchange="ring")


def test_peer_planes_global_range_equal_planes_is_the_round_robin():
    """Equal planes: global_range(s, r, G) is ChunkPlan's global chunk s*G + r."""
    planes = sharded.PeerPlanes(2, 3, 10, "cpu")
    plan = sharded.ChunkPlan(3 * 10 * 4, 4, 10)
    for r in range(4):
        assert [planes.global_range(s, r, 4) for s in range(3)] == plan.owned(r)
    with pytest.raises(IndexError):
        planes.global_range(3, 0, 4)
    with pytest.raises(IndexError):
        planes.global_index(0, 0, 4, 10)


def test_peer_planes_checks_round_shapes():
    with pytest.raises(ValueError, match="positive"):
        sharded.PeerPlanes(3, 0, 0, "cpu", sizes=[10, 0])
    planes = sharded.PeerPlanes(3, 2, 10, "cpu")
    with pytest.raises(ValueError, match="w chunks"):
        planes.aggregate_gather_([torch.zeros(10)], reduce=lambda *a: None)


# ---------------------------------------------------------------- GPU leg
def _gpu_worker(rank, world, port, n, k, rule, chunk, overlap, q, exchange="all_gather"):
    """One rank: the HIP reduce (the default of sharded_aggregate_) on cuda:0,
    gloo for the all-gather (both ranks share the one GPU of the test box;
    the driver's multi-GPU bench uses RCCL)."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        peers = [torch.from_numpy(oracle.synth(n, 23, p, 1e-2)).to(dev) for p in range(k)]
        w = torch.from_numpy(oracle.synth(n, 23, 0xFFFFF, 5e-2)).to(dev)
        plan = sharded_aggregate_(w, peers, rule=rule, chunk=chunk, overlap=overlap, exchange=exchange)
        torch.cuda.synchronize()
        q.put((rank, w.cpu().numpy().tobytes(), plan.full_rounds, plan.tail))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # report, do not hang the parent
        q.put((rank, repr(e), -1, -1))
        raise


@pytest.mark.gpu
@pytest.mark.parametrize("rule,n,k,chunk,overlap,exchange", [
    ("fedavg", 100_003, 9, 8192, True, "all_gather"),  # 6 full rounds + ragged tail, gather on a comm stream
    ("fedavg", 100_003, 64, 8192, True, "p2p"),        # the direct exchange (host-staged on gloo)
    ("median", 40_003, 256, 4096, False, "p2p"),
    ("fedavg", 65_536, 256, 16_384, False, "all_gather"),  # no tail, K = 256
    ("median", 50_001, 130, 4096, True, "all_gather"),    # LDS-staged robust kernel (K > 128)
    ("trimmed", 50_001, 64, 6000, True, "all_gather"),    # one-lane robust kernel, unaligned chunk starts
    ("trimmed", 30_011, 256, 4096, True, "all_gather"),
    ("median", 40_003, 256, 4096, True, "all_gather"),    # the pair kernel (north-star median of 256)
    ("median", 50_001, 128, 6000, True, "all_gather"),    # cfg4's K, unaligned chunk starts
    ("fedavg_torch_gpu", 70_001, 10, 6000, True, "all_gather"),  # FedAvg as torch runs it on the GPU
])
def test_gpu_world2_hip_reduce_byte_identical_to_oracle(cuda, rule, n, k, chunk, overlap, exchange):
    """VERDICT r01 missing #2: sharded_aggregate_ with the DEFAULT (HIP)
    per-shard reduce -- each rank reduces its round-robin chunks on the GPU,
    the all-gather reassembles -- byte-compared with the CPU oracle on both
    ranks (reference aggregation.py:25-38 is coordinate-wise)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, n, k, rule, chunk, overlap, q, exchange))
             for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, b, rounds, tail = q.get(timeout=180)
        assert isinstance(b, bytes), f"rank {r} failed: {b}"
        got[r] = b
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert rounds >= 1 and (tail > 0) == (n % (2 * chunk) != 0)
    peers = [oracle.synth(n, 23, p, 1e-2) for p in range(k)]
    w = oracle.synth(n, 23, 0xFFFFF, 5e-2)
    if rule in ("fedavg", "fedavg_torch_gpu"):
        want, _ = oracle.fedavg(peers, w, torch_gpu=rule == "fedavg_torch_gpu")
    else:
        rid = 1 if rule == "median" else 2
        want, _ = oracle.robust(peers, rid, oracle.trim_count(k) if rid == 2 else 0, w=w)
    assert got[0] == got[1], "ranks disagree after the all-gather"
    g = np.frombuffer(got[0], dtype=np.uint32)
    bad = np.nonzero(g != want.view(np.uint32))[0]
    assert bad.size == 0, f"{bad.size} coordinates differ, first {bad[:5]}"


# ---------------------------------------------------------------- digests by peer
def _sha_host(msgs):
    import hashlib
    return [hashlib.sha256(m).digest() for m in msgs]


def _messages(k, seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes() for _ in range(k)]


def _digest_worker(rank, world, port, k, use_gpu, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from p2pdl_amd.sharded import sharded_digests

        if use_gpu:
            torch.cuda.set_device(0)
        got = sharded_digests(_messages(k, 5), digest=None if use_gpu else _sha_host)
        q.put((rank, got))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # report, do not hang the parent
        q.put((rank, repr(e)))
        raise


def _run_digest_world(world, k, use_gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_digest_worker, args=(r, world, port, k, use_gpu, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, d = q.get(timeout=180)
        assert isinstance(d, list), f"rank {r} failed: {d}"
        got[r] = d
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    want = _sha_host(_messages(k, 5))
    for r in range(world):
        assert got[r] == want, f"rank {r}"


@pytest.mark.parametrize("world,k", [(2, 7), (2, 1), (3, 10)])
def test_digests_sharded_by_peer_gloo(world, k):
    """§8(e) digest row: message j hashed on rank j % G, one all-gather of the
    32-B digests; every rank ends with all K digests in list order (here with
    the host hash through the test seam; the GPU leg below uses the kernel)."""
    _run_digest_world(world, k, use_gpu=False)


@pytest.mark.gpu
def test_digests_sharded_by_peer_gpu_kernel(cuda):
    """The same with the HIP SHA-256 batch kernel on every rank (both ranks
    on cuda:0, gloo for the gather), against hashlib."""
    _run_digest_world(2, 9, use_gpu=True)


def _nccl_world1_worker(port, q):
    """World 1 over the real backend (RCCL): sharded_aggregate_ still issues
    its all_gather_into_tensor calls (in place), so the RCCL call path of the
    multi-GPU reduce runs on the one-GPU box."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        out = {}
        for rule, n, k, chunk in [("median", 40_003, 256, 4096), ("fedavg", 100_003, 9, 8192)]:
            peers = [torch.from_numpy(oracle.synth(n, 29, p, 1e-2)).to(dev) for p in range(k)]
            w = torch.from_numpy(oracle.synth(n, 29, 0xFFFFF, 5e-2)).to(dev)
            sharded_aggregate_(w, peers, rule=rule, chunk=chunk)
            torch.cuda.synchronize()
            out[rule] = (w.cpu().numpy().tobytes(), dist.get_backend())
        # the memory-sharded plane round: HIP reduce per plane, each plane's
        # RCCL all-gather on a second stream beside the next plane
        k, S, C = 20, 3, 70_001
        planes = sharded.PeerPlanes(k, S, C, dev)
        peers = [oracle.synth(S * C, 37, p, 1e-2) for p in range(k)]
        w = oracle.synth(S * C, 37, 0xFFFFF, 5e-2)
        for s_ in range(S):
            for p in range(k):
                planes.row(s_, p).copy_(torch.from_numpy(peers[p][s_ * C:(s_ + 1) * C]))
        ws = [torch.from_numpy(w[s_ * C:(s_ + 1) * C].copy()).to(dev) for s_ in range(S)]
        w_full = torch.zeros(S * C, dtype=torch.float32, device=dev)
        planes.aggregate_gather_(ws, w_full, rule="fedavg", comm=torch.cuda.Stream(dev))
        torch.cuda.synchronize()
        out["planes"] = (w_full.cpu().numpy().tobytes(), dist.get_backend())
        # the direct exchange's call path (at world 1: the own piece only)
        ws = [torch.from_numpy(w[s_ * C:(s_ + 1) * C].copy()).to(dev) for s_ in range(S)]
        w_full.zero_()
        planes.aggregate_gather_(ws, w_full, rule="fedavg", comm=torch.cuda.Stream(dev), exchange="p2p")
        torch.cuda.synchronize()
        out["planes_p2p"] = (w_full.cpu().numpy().tobytes(), dist.get_backend())
        q.put(out)
        dist.destroy_process_group()
    except BaseException as e:  # report, do not hang the parent
        q.put(repr(e))
        raise


@pytest.mark.gpu
def test_gpu_world1_nccl_allgather_path(cuda):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_world1_worker, args=(_free_port(), q))
    p.start()
    got = q.get(timeout=180)
    p.join(60)
    assert isinstance(got, dict), got
    assert p.exitcode == 0
    for rule, n, k in [("median", 40_003, 256), ("fedavg", 100_003, 9)]:
        b, backend = got[rule]
        assert backend == "nccl"
        peers = [oracle.synth(n, 29, p, 1e-2) for p in range(k)]
        w = oracle.synth(n, 29, 0xFFFFF, 5e-2)
        want = oracle.fedavg(peers, w)[0] if rule == "fedavg" else oracle.robust(peers, 1, 0, w=w)[0]
        assert b == want.tobytes(), rule
    b, backend = got["planes"]
    peers = [oracle.synth(3 * 70_001, 37, p, 1e-2) for p in range(20)]
    want = oracle.fedavg(peers, oracle.synth(3 * 70_001, 37, 0xFFFFF, 5e-2))[0].tobytes()
    assert backend == "nccl" and b == want
    assert got["planes_p2p"] == (want, "nccl")


def _subgroup_exchange_worker(rank, world, port, q):
    """exchange_ over a process subgroup: group ranks map to global ranks."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        members = [0, 2]
        grp = dist.new_group(members)  # every rank takes part in new_group
        got = None
        if rank in members:
            C, r = 5, members.index(rank)
            mine = torch.arange(C, dtype=torch.float32) + 100 * rank
            for kind in sharded.EXCHANGES:
                out = torch.full((2 * C,), -1.0)
                sharded.exchange_(out, mine, grp, kind)
                got = (got or {}) | {kind: out.tolist()}
            assert r == members.index(rank)
        q.put((rank, got))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_exchange_over_a_subgroup():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_subgroup_exchange_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    want = [float(i) for i in range(5)] + [200.0 + i for i in range(5)]
    assert got[1] is None
    for r in (0, 2):
        assert got[r] == {"all_gather": want, "p2p": want}
