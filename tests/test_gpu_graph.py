"""The C ABI's calls are stream-ordered, allocate nothing and keep no state
(include/p2pdl.h), so they can be captured into a HIP graph and replayed
(INTEGRATION.md §2): captured once, replayed three times, every kernel
family gives the bits of three eager calls -- FedAvg (reference
aggregator/aggregation.py:15-38), the robust rules at K = 64 / 128 / 256 and
the trainer delta (node/node.py:273-282)."""
import numpy as np
import pytest
import torch

import oracle


def _dev(a, cuda):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(cuda)


@pytest.mark.gpu
def test_fedavg_graph_replay_equals_repeated_calls(cuda):
    from p2pdl_amd import ops

    k, n = 5, 100_003
    peers = [oracle.synth(n, 31, p, 1e-2) for p in range(k)]
    w0 = oracle.synth(n, 31, 0xFFFFF, 5e-2)
    pd = [_dev(p, cuda) for p in peers]
    table = ops.pointer_table(pd, cuda)  # device table built before the capture
    w = _dev(w0, cuda)
    ops.aggregate(None, "fedavg", w=w, lr=0.1, table=table)  # warm-up
    torch.cuda.synchronize()
    w.copy_(_dev(w0, cuda))
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(cuda)
    s.wait_stream(torch.cuda.current_stream(cuda))
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            ops.aggregate(None, "fedavg", w=w, lr=0.1, table=table)
    torch.cuda.synchronize()
    assert np.array_equal(w.cpu().numpy().view(np.uint32), w0.view(np.uint32)), "capture must not execute"
    want = w0
    for _ in range(3):
        g.replay()
        want, _ = oracle.fedavg(peers, want)
    torch.cuda.synchronize()
    assert np.array_equal(w.cpu().numpy().view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("rule,k", [("median", 64), ("trimmed", 128), ("median", 256), ("trimmed", 256)])
def test_robust_graph_replay(cuda, rule, k):
    from p2pdl_amd import ops

    n = 20_011
    peers = [oracle.synth(n, 37, p, 1e-2) for p in range(k)]
    w0 = oracle.synth(n, 37, 0xFFFFF, 5e-2)
    keep = [_dev(p, cuda) for p in peers]  # the table's targets stay alive
    table = ops.pointer_table(keep, cuda)
    w = _dev(w0, cuda)
    ops.aggregate(None, rule, w=w, lr=0.1, table=table)  # warm-up
    torch.cuda.synchronize()
    w.copy_(_dev(w0, cuda))
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(cuda)
    s.wait_stream(torch.cuda.current_stream(cuda))
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            ops.aggregate(None, rule, w=w, lr=0.1, table=table)
    rid = ops.rule_id(rule)
    b = ops.trim_count(k) if rid == 2 else 0
    want = w0
    for _ in range(3):
        g.replay()
        want, _ = oracle.robust(peers, rid, b, w=want)
    torch.cuda.synchronize()
    assert np.array_equal(w.cpu().numpy().view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
def test_delta_graph_replay(cuda):
    """Two replays of one captured delta launch: prev follows cur, delta is
    cur - prev of the previous replay (0 after the first)."""
    from p2pdl_amd import ops

    n = 70_001
    c0, p0 = oracle.synth(n, 41, 1, 1e-1), oracle.synth(n, 41, 2, 1e-1)
    cur, prev = _dev(c0, cuda), _dev(p0, cuda)
    delta = torch.empty_like(cur)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(cuda)
    s.wait_stream(torch.cuda.current_stream(cuda))
    ops.delta_snapshot_(cur, torch.empty_like(cur), delta, first=True)  # warm-up (other buffers)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            ops.delta_snapshot_(cur, prev, delta)
    g.replay()
    torch.cuda.synchronize()
    want, _ = oracle.delta_snapshot_np(c0, p0)
    assert np.array_equal(delta.cpu().numpy().view(np.uint32), want.view(np.uint32))
    assert torch.equal(prev, cur)
    g.replay()
    torch.cuda.synchronize()
    assert not delta.cpu().numpy().view(np.uint32).any()  # x - x = +0 for every finite x


@pytest.mark.gpu
@pytest.mark.parametrize("route", ["flat", "chunks"])
def test_split_kernel_graph_replay(cuda, route):
    """The LDS-DMA split kernel captured and replayed (K = 16, more than one
    round of tiles): a flat buffer, and a state_dict of separately allocated
    tensors on the chunk list (its device table built before the capture).
    A build with the tile queue keeps one counter pair per captured launch,
    so the replays run in order on it."""
    from p2pdl_amd import ops

    k = 16
    sizes = [256 * 8192 + 4099] if route == "flat" else [1_234_567, 5, 1_000_003]
    peers = [[oracle.synth(n, 41 + i, p, 1e-2) for i, n in enumerate(sizes)] for p in range(k)]
    w0 = [oracle.synth(n, 41 + i, 0xFFFFF, 5e-2) for i, n in enumerate(sizes)]
    pd = [[_dev(a, cuda) for a in row] for row in peers]
    ws = [_dev(a, cuda) for a in w0]
    if route == "flat":
        table = ops.pointer_table([row[0] for row in pd], cuda)
        run = lambda: ops.aggregate(None, "fedavg", w=ws[0], lr=0.1, table=table)  # noqa: E731
    else:
        ptrs = np.array([[row[i].data_ptr() for row in pd] for i in range(len(sizes))], dtype=np.uint64)
        ops.aggregate_ptr_table_(ws, ptrs, "fedavg")  # builds and caches the device table
        entry = next(reversed(ops._TABLES.values()))
        assert entry[5][2][3] == "chunks"
        run = lambda: ops._launch_entry(entry, k, 0.1, ops.N.stream_handle())  # noqa: E731
    run()  # warm-up
    torch.cuda.synchronize()
    for w, a in zip(ws, w0):
        w.copy_(_dev(a, cuda))
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(cuda)
    s.wait_stream(torch.cuda.current_stream(cuda))
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            run()
    want = list(w0)
    for _ in range(3):
        g.replay()
        want = [oracle.fedavg([row[i] for row in peers], want[i])[0] for i in range(len(sizes))]
    torch.cuda.synchronize()
    for w, a in zip(ws, want):
        assert np.array_equal(w.cpu().numpy().view(np.uint32), a.view(np.uint32))


@pytest.mark.gpu
def test_captured_split_launch_keeps_its_queue_pair(cuda):
    """A captured split launch owns its tile-queue counter pair (fedavg.hip
    queue_slot): its replays on one stream, overlapping 4,200 ordinary split
    launches on another -- more than the rotating pairs, so each of those
    pairs is reused -- never share a counter with them.  Every output is
    poisoned before its launch and compared on the device after it: a launch
    that lost tiles to another's claims would leave NaNs behind.  FedAvg
    mean (reference aggregator/aggregation.py:25-32), K = 16 over 300 whole
    split tiles (> one per CU: the persistent grid claims tiles)."""
    from p2pdl_amd import ops

    k, n, iters = 16, 300 * 8192, 4200
    peers = [oracle.synth(n, 83, p, 1e-2) for p in range(k)]
    _, mean = oracle.fedavg(peers)
    pd = [_dev(p, cuda) for p in peers]  # kept alive: the table holds only their addresses
    table = ops.pointer_table(pd, cuda)
    want = _dev(mean, cuda).view(torch.int32)
    sa, sb = torch.cuda.Stream(cuda), torch.cuda.Stream(cuda)
    out_a = torch.empty(n, dtype=torch.float32, device=cuda)
    out_b = torch.empty_like(out_a)
    ops.aggregate(None, "fedavg", out=out_a, table=table)  # warm-up
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    sa.wait_stream(torch.cuda.current_stream(cuda))
    with torch.cuda.stream(sa):
        with torch.cuda.graph(g, stream=sa):
            ops.aggregate(None, "fedavg", out=out_a, table=table)
    torch.cuda.synchronize()
    bad_a = torch.zeros((), dtype=torch.int64, device=cuda)
    bad_b = torch.zeros_like(bad_a)
    main = torch.cuda.current_stream(cuda)
    for i in range(iters):
        if i % 600 == 0:  # progress (and a bounded queue) for the run's hang guard
            torch.cuda.synchronize()
            print(f"captured-pair test: {i} / {iters}", flush=True)
        # fork / join: both launches of an iteration start together, so the
        # one that would share a pair overlaps the replay
        sa.wait_stream(main)
        sb.wait_stream(main)
        with torch.cuda.stream(sa):
            out_a.fill_(float("nan"))
            g.replay()
            bad_a += (out_a.view(torch.int32) != want).sum()
        with torch.cuda.stream(sb):
            out_b.fill_(float("nan"))
            ops.aggregate(None, "fedavg", out=out_b, table=table)
            bad_b += (out_b.view(torch.int32) != want).sum()
        main.wait_stream(sa)
        main.wait_stream(sb)
    torch.cuda.synchronize()
    assert int(bad_a) == 0 and int(bad_b) == 0, (int(bad_a), int(bad_b))
    del pd
