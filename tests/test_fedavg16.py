"""FedAvg on float16 / bfloat16 models (reference aggregator/aggregation.py:
15-38 on a half-precision state_dict; ops.fedavg16_apply_, include/p2pdl.h
p2p_fedavg_apply_16).  torch runs each op in fp32 and rounds to the storage
type; the oracle (oracle.fedavg16_np) restates that and is pinned to the
reference's own aggregate_models run on CPU (tests/golden/make_golden_16.py
-> fedavg16_golden.npz: MLP K=3, ragged K=7, K=10, special values).  On the
GPU: the kernel against the goldens, the drop-in on a half model, the
reference's ops run by torch on the GPU against the oracle's torch_gpu mode
and the kernel's fedavg_torch_gpu rule, and the error paths."""
import hashlib
import json
import os
import types

import numpy as np
import pytest
import torch

import oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden", "fedavg16_golden.npz")
TDT = {"float16": torch.float16, "bfloat16": torch.bfloat16}
W_PEER, W_SCALE, UPD_SCALE = 0xFFFFF, 5e-2, 1e-2


def _cases():
    z = np.load(GOLD)  # allow_pickle=False (default): data only
    return z, json.loads(bytes(z["meta"]).decode())["cases"]


def _inputs(z, c):
    key = f"{c['dtype']}__{c['name']}"
    n = sum(int(np.prod(s)) for _, s in c["shapes"])
    if f"{key}__w" in z.files:
        return z[f"{key}__w"], [z[f"{key}__peer{i}"] for i in range(c["k"])], z[f"{key}__out"]
    w = oracle.round_16(oracle.synth_np(n, c["seed"], W_PEER, W_SCALE), c["dtype"])
    peers = [oracle.round_16(oracle.synth_np(n, c["seed"], p, UPD_SCALE), c["dtype"]) for p in range(c["k"])]
    return w, peers, None


def _same(a, b, dtype):
    fa, fb = oracle.to_f32_16(a, dtype), oracle.to_f32_16(b, dtype)
    return bool(np.all((np.isnan(fa) & np.isnan(fb)) | (np.asarray(a) == np.asarray(b))))


def _check(got, c, out):
    if out is not None:
        assert _same(got, out, c["dtype"]), f"{c['dtype']} {c['name']}"
    else:
        assert hashlib.sha256(np.ascontiguousarray(got).tobytes()).hexdigest() == c["out_sha256"], c["name"]


def test_oracle_matches_the_reference_on_16_bit_models():
    z, cases = _cases()
    assert {c["dtype"] for c in cases} == {"float16", "bfloat16"} and len(cases) == 8
    for c in cases:
        w, peers, out = _inputs(z, c)
        _check(oracle.fedavg16_np(peers, w, c["dtype"]), c, out)


def test_rounding_helpers_match_torch():
    rng = np.random.default_rng(3)
    x = np.concatenate([(rng.standard_normal(50_000) * 10).astype(np.float32),
                        np.array([0.0, -0.0, np.inf, -np.inf, 1e-40, 65519.0, 65520.0, 3.4e38], np.float32)])
    for dt, tdt in TDT.items():
        bits = torch.from_numpy(x).to(tdt).view(torch.int16).numpy().view(np.uint16)
        assert np.array_equal(oracle.round_16(x, dt), bits), dt
        assert np.array_equal(oracle.to_f32_16(bits, dt), torch.from_numpy(x).to(tdt).float().numpy()), dt


# ----------------------------------------------------------------- GPU
def _dev16(bits, dt, dev, shape=None):
    t = torch.from_numpy(np.ascontiguousarray(bits, dtype=np.uint16).view(np.int16).copy()).view(TDT[dt]).to(dev)
    return t.reshape(shape) if shape is not None else t


def _host16(t):
    torch.cuda.synchronize()
    return t.detach().contiguous().view(torch.int16).cpu().numpy().view(np.uint16).reshape(-1)


@pytest.mark.gpu
@pytest.mark.parametrize("rule", ["fedavg", "fedavg_torch_gpu"])
def test_kernel_matches_goldens_and_oracle(cuda, rule):
    from p2pdl_amd import ops

    z, cases = _cases()
    for c in cases:
        w, peers, out = _inputs(z, c)
        wt = _dev16(w, c["dtype"], cuda)
        ops.fedavg16_apply_(wt, [_dev16(p, c["dtype"], cuda) for p in peers], rule)
        got = _host16(wt)
        want = oracle.fedavg16_np(peers, w, c["dtype"], torch_gpu=rule == "fedavg_torch_gpu")
        assert _same(got, want, c["dtype"]), f"{rule} {c['dtype']} {c['name']} vs oracle"
        if rule == "fedavg":
            _check(got, c, out)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", ["float16", "bfloat16"])
@pytest.mark.parametrize("shift", [0, 1, 2, 3])
def test_misaligned_and_ragged(cuda, dt, shift):
    """Views 2*shift bytes off an 8-byte boundary (the element path) and
    lengths that are not a multiple of 4."""
    from p2pdl_amd import ops

    k, n = 5, 4097
    w = oracle.round_16(oracle.synth_np(n, 77 + shift, W_PEER, W_SCALE), dt)
    peers = [oracle.round_16(oracle.synth_np(n, 77 + shift, p, UPD_SCALE), dt) for p in range(k)]
    base = [torch.zeros(n + 4, dtype=TDT[dt], device=cuda) for _ in range(k + 1)]
    wt = base[0][shift:shift + n]
    wt.copy_(_dev16(w, dt, cuda))
    pt = []
    for b, p in zip(base[1:], peers):
        b[shift:shift + n].copy_(_dev16(p, dt, cuda))
        pt.append(b[shift:shift + n])
    ops.fedavg16_apply_(wt, pt)
    assert _same(_host16(wt), oracle.fedavg16_np(peers, w, dt), dt)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", ["float16", "bfloat16"])
@pytest.mark.parametrize("rule", ["fedavg", "fedavg_torch_gpu"])
def test_drop_in_on_a_half_model(cuda, dt, rule, monkeypatch):
    """aggregate_models on a model.half()-style MLP: the golden MLP case
    (the reference's own result on CPU) and, for the GPU rule, the
    reference's ops run by torch on this GPU."""
    from p2pdl_amd.aggregator import aggregation as agg

    monkeypatch.setattr(agg, "broadcast_global_model_update", lambda self: None)
    z, cases = _cases()
    c = next(c for c in cases if c["dtype"] == dt and c["name"] == "mlp_k3")
    w, peers, _ = _inputs(z, c)
    shapes = [(nm.replace(".", "__"), tuple(s)) for nm, s in c["shapes"]]

    def split(bits):
        out, o = {}, 0
        for nm, s in shapes:
            n = int(np.prod(s))
            out[nm] = _dev16(bits[o:o + n], dt, cuda, s)
            o += n
        return out

    model = torch.nn.Module()
    for nm, t in split(w).items():
        model.register_parameter(nm, torch.nn.Parameter(t, requires_grad=False))
    ups = [split(p) for p in peers]
    node = types.SimpleNamespace(model=model, received_models=[{"model": u} for u in ups], trainers_list=[0] * 3,
                                 addr="a", port=1, neighbors=[])
    agg.aggregate_models(node, rule=rule)
    got = np.concatenate([_host16(t) for t in model.state_dict().values()])
    assert node.received_models == []
    if rule == "fedavg":
        _check(got, c, None)
        return
    state = split(w)  # the reference's loop (aggregation.py:15-38) in torch on this GPU
    acc = {k: torch.zeros_like(v) for k, v in state.items()}
    for u in ups:
        for k in acc:
            acc[k] += u[k]
    for k in acc:
        acc[k] /= 3
    for k in state:
        state[k] += 0.1 * acc[k]
    live = np.concatenate([_host16(t) for t in state.values()])
    want = oracle.fedavg16_np(peers, w, dt, torch_gpu=True)
    assert _same(got, want, dt), "kernel vs oracle"
    if dt == "bfloat16":
        assert _same(live, want, dt), "torch on the GPU vs oracle"
        return
    # float16: torch's vectorized GPU path rounds every op fp32-then-f16 like
    # the oracle; where its elementwise kernel takes the non-vectorized path
    # (seen on the 2,560-element fc3 weight) the compiled mul single-rounds
    # lr * acc (v_fma_mixlo_f16), so the few coordinates whose fp32 product
    # lands on an f16 midpoint differ there -- each must be exactly that
    off = np.nonzero(live != want)[0]
    assert off.size <= 16, off.size
    f = lambda b: oracle.to_f32_16(b, dt)
    s_ = np.zeros(live.size, np.float32)
    for p in peers:
        s_ = f(oracle.round_16(s_ + f(p), dt))
    m = f(oracle.round_16(s_ * (np.float32(1.0) / np.float32(3)), dt))
    t_once = f(oracle.round_16_once(np.float64(np.float32(0.1)) * m[off].astype(np.float64), dt))
    assert np.array_equal(live[off], oracle.round_16(f(w[off]) + t_once, dt)), "torch's tail rounding"


@pytest.mark.gpu
def test_16_bit_error_paths(cuda, monkeypatch):
    from p2pdl_amd.aggregator import aggregation as agg

    monkeypatch.setattr(agg, "broadcast_global_model_update", lambda self: None)

    def node(model, ups):
        return types.SimpleNamespace(model=model, received_models=[{"model": u} for u in ups],
                                     trainers_list=[0] * len(ups), addr="a", port=1, neighbors=[])

    m = torch.nn.Linear(4, 3).to(cuda).half()
    good = {k: v.clone() for k, v in m.state_dict().items()}
    with pytest.raises(NotImplementedError):
        agg.aggregate_models(node(m, [good]), rule="median")
    with pytest.raises(NotImplementedError):
        agg.aggregate_models(node(m, [{k: v.float() for k, v in good.items()}]))
    with pytest.raises(KeyError):
        agg.aggregate_models(node(m, [{"weight": good["weight"]}]))
    mixed = torch.nn.Linear(4, 3).to(cuda).half()
    mixed.bias.data = mixed.bias.data.float()
    with pytest.raises(NotImplementedError):
        agg.aggregate_models(node(mixed, [{k: v.clone() for k, v in mixed.state_dict().items()}]))
    bn = torch.nn.BatchNorm1d(3).to(cuda).half()  # int64 num_batches_tracked: the reference fails at :32
    with pytest.raises(RuntimeError, match="Long"):
        agg.aggregate_models(node(bn, [{k: v.clone() for k, v in bn.state_dict().items()}]))
    assert torch.equal(m.weight, good["weight"])  # nothing was applied
