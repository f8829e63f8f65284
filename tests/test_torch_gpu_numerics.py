"""FedAvg bit-exact with the reference AS DEPLOYED -- its ops run by torch on
GPU tensors (reference node/node.py:28-29 puts the model on cuda) -- the
product's ``fedavg_torch_gpu`` rule (include/p2pdl.h P2P_RULE_FEDAVG_TORCH_GPU).

On a GPU tensor ATen divides by the CPU scalar K (aggregation.py:32) as a
multiply by fl(1/K); the CPU reference (the default rule, the goldens of
make_golden.py) divides.  Pinning, in order:
  * the oracle's torch_gpu mode against ``tests/golden/fedavg_torch_gpu.npz``,
    written on an MI355X by ``make_golden_torch_gpu.py`` (the reference's op
    sequence in torch on the GPU) -- CPU test;
  * the same op sequence run live in torch on this box's GPU against the
    oracle, then the HIP kernels (flat, segment table, drop-in
    ``aggregate_models``, misaligned views) against both -- GPU tests.
"""
import hashlib
import importlib.util
import json
import os
import types

import numpy as np
import pytest
import torch

import oracle

_GEN = os.path.join(os.path.dirname(__file__), "golden", "make_golden_torch_gpu.py")
_spec = importlib.util.spec_from_file_location("make_golden_torch_gpu", _GEN)
G = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(G)  # the fixture's generator: case list and the reference's op sequence

FIXTURE = os.path.join(os.path.dirname(__file__), "golden", "fedavg_torch_gpu.npz")


def _fixture():
    z = np.load(FIXTURE)  # allow_pickle=False (default): data only
    meta = json.loads(bytes(z["meta"]).decode())
    return z, meta


def _oracle_case(K, shapes, seed, torch_gpu):
    w, peers = G.inputs(K, [(n, tuple(s)) for n, s in shapes], seed)
    return oracle.fedavg(peers, w, torch_gpu=torch_gpu)[0]


def test_oracle_torch_gpu_mode_matches_the_mi355x_fixture():
    z, meta = _fixture()
    assert [c["name"] for c in meta["cases"]] == [c[0] for c in G.CASES]
    for c in meta["cases"]:
        got = _oracle_case(c["k"], c["shapes"], c["seed"], True)
        assert hashlib.sha256(got.tobytes()).hexdigest() == c["sha256"], c["name"]
        if c["name"] in z.files:
            assert np.array_equal(got.view(np.uint32), z[c["name"]].view(np.uint32)), c["name"]
        cpu = _oracle_case(c["k"], c["shapes"], c["seed"], False)
        if c["k"] & (c["k"] - 1):  # K not a power of two: 1/K inexact, the two references differ
            assert not np.array_equal(cpu, got), c["name"]
        else:  # K = 2^j: x * 2^-j == x / 2^j exactly
            assert np.array_equal(cpu.view(np.uint32), got.view(np.uint32)), c["name"]


def test_rule_name_and_tile():
    from p2pdl_amd import ops

    assert ops.rule_id("fedavg_torch_gpu") == 3 and ops.rule_id(3) == 3
    assert 3 in ops.FEDAVG_RULES


# ----------------------------------------------------------------- GPU
def _flat(case, dev):
    name, K, shapes, seed = case
    w, peers = G.inputs(K, shapes, seed)
    return (torch.from_numpy(w).to(dev), [torch.from_numpy(p).to(dev) for p in peers], w, peers)


@pytest.mark.gpu
@pytest.mark.parametrize("case", G.CASES, ids=[c[0] for c in G.CASES])
def test_live_torch_gpu_ops_equal_oracle_and_kernel(cuda, case):
    from p2pdl_amd import ops

    name, K, shapes, seed = case
    live = G.reference_ops_on(cuda, K, shapes, seed)  # the reference's ops, torch on this GPU
    want = _oracle_case(K, [(n, list(s)) for n, s in shapes], seed, True)
    assert np.array_equal(live.view(np.uint32), want.view(np.uint32)), "torch on the GPU vs oracle"
    wt, pt, _, _ = _flat(case, cuda)
    ops.aggregate(pt, "fedavg_torch_gpu", w=wt, lr=0.1)
    torch.cuda.synchronize()
    assert np.array_equal(wt.cpu().numpy().view(np.uint32), want.view(np.uint32)), "flat kernel"
    z, meta = _fixture()
    rec = {c["name"]: c for c in meta["cases"]}[name]
    assert hashlib.sha256(live.tobytes()).hexdigest() == rec["sha256"], "this box vs the fixture's box"


@pytest.mark.gpu
def test_drop_in_aggregate_models_torch_gpu_rule(cuda):
    """aggregate_models(node, rule='fedavg_torch_gpu') on a cuda model:
    bit-exact with the reference's ops run by torch on the GPU, through the
    C-gathered table (contiguous updates) and the per-tensor segment path (a
    transposed update view)."""
    from p2pdl_amd.aggregator import aggregation as agg

    name, K, shapes, seed = G.CASES[1]  # ragged_k7
    want = G.reference_ops_on(cuda, K, shapes, seed)
    for transposed in (False, True):
        w, peers = G.inputs(K, shapes, seed)
        model = torch.nn.Module()
        for nm, t in G.split(w, shapes, cuda).items():
            model.register_parameter(nm, torch.nn.Parameter(t, requires_grad=False))
        ups = [G.split(p, shapes, cuda) for p in peers]
        if transposed:
            ups[2] = dict(ups[2])
            ups[2]["a"] = ups[2]["a"].t().contiguous().t()  # same values, non-contiguous view
            assert not ups[2]["a"].is_contiguous()
        node = types.SimpleNamespace(model=model, received_models=[{"model": u} for u in ups],
                                     trainers_list=[0] * K, addr="127.0.0.1", port=7000, neighbors=[])
        orig = agg.broadcast_global_model_update
        agg.broadcast_global_model_update = lambda self: None
        try:
            agg.aggregate_models(node, rule="fedavg_torch_gpu")
        finally:
            agg.broadcast_global_model_update = orig
        got = np.concatenate([t.detach().cpu().numpy().reshape(-1) for t in model.state_dict().values()])
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"transposed={transposed}"
        assert node.received_models == []


@pytest.mark.gpu
@pytest.mark.parametrize("shift", [1, 2, 3])
def test_misaligned_views_take_the_element_path(cuda, shift):
    """Views 4*shift bytes off a 16-B boundary: the element-wise kernel path,
    same division form."""
    from p2pdl_amd import ops

    K, n = 10, 4099
    w, peers = G.inputs(K, [("x", (n,))], 0x5EED1010 + shift)
    base = [torch.zeros(n + 4, device=cuda) for _ in range(K + 1)]
    wt = base[0][shift:shift + n]
    wt.copy_(torch.from_numpy(w))
    pt = []
    for b, p in zip(base[1:], peers):
        v = b[shift:shift + n]
        v.copy_(torch.from_numpy(p))
        pt.append(v)
    ops.aggregate(pt, "fedavg_torch_gpu", w=wt, lr=0.1)
    torch.cuda.synchronize()
    want = oracle.fedavg(peers, w, torch_gpu=True)[0]
    assert np.array_equal(wt.cpu().numpy().view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("K", [3, 7, 64])
def test_special_values_match_torch_on_the_gpu(cuda, K):
    """±0, subnormals, ±inf, NaN and overflow through the reference's ops run
    by torch on the GPU, against the kernel's fedavg_torch_gpu rule and the
    oracle: subnormal inputs, quotients and products are kept (no flush to
    zero on either side), NaN compared as a class."""
    from p2pdl_amd import ops

    rng = np.random.default_rng(7 + K)
    tiny = np.array([0.0, -0.0, 1e-45, -1e-45, 1.17e-38, -3e-39, 2e-39, 5e-39, -7e-40], dtype=np.float32)
    sp = np.array([np.inf, -np.inf, np.nan, 3.4e38, -3.4e38, 1.0, -1.0, 1e-7, 0.1, 1 / 3, 5e-38], dtype=np.float32)
    n = 4099

    def draw():  # mostly zeros and subnormals, specials at ~1 in 300 positions
        x = rng.choice(tiny, size=n).astype(np.float32)
        hit = rng.random(n) < 1 / 300
        x[hit] = rng.choice(sp, size=int(hit.sum()))
        return x

    peers = [draw() for _ in range(K)]
    w0 = draw()
    # the reference's loop (aggregation.py:15-38) in torch on the GPU
    acc = torch.zeros(n, device=cuda)
    for p in peers:
        acc += torch.from_numpy(p).to(cuda)
    acc /= K
    wt_ref = torch.from_numpy(w0.copy()).to(cuda)
    wt_ref += 0.1 * acc
    live = wt_ref.cpu().numpy()
    want = oracle.fedavg(peers, w0, torch_gpu=True)[0]
    wt = torch.from_numpy(w0.copy()).to(cuda)
    ops.aggregate([torch.from_numpy(p).to(cuda) for p in peers], "fedavg_torch_gpu", w=wt, lr=0.1)
    got = wt.cpu().numpy()

    def same(a, b):
        nan = np.isnan(a) & np.isnan(b)
        return bool(np.all(nan | (a.view(np.uint32) == b.view(np.uint32))))

    assert same(live, want), "torch on the GPU vs the oracle"
    assert same(got, live), "kernel vs torch on the GPU"
    assert np.any((np.abs(live) < 1.18e-38) & (live != 0)), "the case holds subnormal results"
