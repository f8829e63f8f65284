#!/usr/bin/env python3
"""Generate golden FedAvg vectors by running the REFERENCE aggregator.

Runs only in the build container (it needs /root/reference, which never
travels to the GPU box).  It imports the reference's own
``aggregator/aggregation.py::aggregate_models`` (reference :7-46) through the
harness of SURVEY.md §8(c): /root/reference is symlinked as package ``p2pdl``
under a temp dir, ``broadcast_global_model_update`` is monkeypatched to a
no-op (it would open TCP sockets, reference :66-77), and the function is called
with a fake Node exactly as ``node/node.py:316`` calls it.

Inputs come from the build's counter PRNG (numpy restatement in
``oracle.synth_np``), so a test can regenerate any input from its seed.  What is
committed: ``fedavg_golden.json`` (case specs, SHA-256 of every output,
strided output samples, behaviour of the error paths) and ``fedavg_small.npz``
(full inputs and outputs of the small / special-value cases).

Usage:  python tests/golden/make_golden.py   (from the repo root)
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
import oracle  # noqa: E402  (test infrastructure: PRNG restatement only)

REF = "/root/reference"
W_PEER = 0xFFFFF  # PRNG stream id used for the model weights
UPD_SCALE, W_SCALE = 1e-2, 5e-2

MLP_SHAPES = [("fc1.weight", (512, 784)), ("fc1.bias", (512,)), ("fc2.weight", (256, 512)),
              ("fc2.bias", (256,)), ("fc3.weight", (10, 256)), ("fc3.bias", (10,))]


def import_reference():
    tmp = tempfile.mkdtemp(prefix="p2pdl_ref_")
    os.symlink(REF, os.path.join(tmp, "p2pdl"))
    sys.path.insert(0, tmp)
    import p2pdl.aggregator.aggregation as agg  # the reference module
    agg.broadcast_global_model_update = lambda self: None
    return agg


class Holder(torch.nn.Module):
    """Module whose state_dict has exactly the given (name, shape) tensors."""

    def __init__(self, shapes, dtypes=None):
        super().__init__()
        self._names = []
        for idx, (name, shape) in enumerate(shapes):
            dt = (dtypes or {}).get(name, torch.float32)
            safe = name.replace(".", "__")
            if dt.is_floating_point:
                self.register_parameter(safe, torch.nn.Parameter(torch.zeros(shape, dtype=dt)))
            else:
                self.register_buffer(safe, torch.zeros(shape, dtype=dt))
            self._names.append(safe)


def flat_split(vec, shapes):
    out, o = {}, 0
    for name, shape in shapes:
        n = int(np.prod(shape))
        out[name.replace(".", "__")] = torch.from_numpy(vec[o:o + n].reshape(shape).copy())
        o += n
    return out


def run_ref(agg, shapes, w_flat, peer_flats):
    model = Holder(shapes)
    with torch.no_grad():
        model.load_state_dict(flat_split(w_flat, shapes))
    recv = [{"model": flat_split(p, shapes), "sender": ("127.0.0.1", 7001 + i)}
            for i, p in enumerate(peer_flats)]
    node = types.SimpleNamespace(model=model, received_models=recv, trainers_list=[0] * len(recv),
                                 addr="127.0.0.1", port=7000, neighbors=[])
    agg.aggregate_models(node)
    assert node.received_models == []  # reference :43
    return np.concatenate([t.detach().numpy().reshape(-1) for t in model.state_dict().values()])


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float32).tobytes()).hexdigest()


def special_case():
    """K=4 peers x 64 coords covering +-0, subnormals, +-inf, NaN and overflow."""
    rng = np.random.default_rng(20241022)
    sp = np.array([0.0, -0.0, 1e-45, -1e-45, 1.17e-38, -3e-39, np.inf, -np.inf, np.nan,
                   3.4e38, -3.4e38, 1.0, -1.0, 1e-7, 0.1, 1 / 3], dtype=np.float32)
    peers = [rng.choice(sp, size=64).astype(np.float32) for _ in range(4)]
    peers[0][:8] = -0.0  # all-negative-zero columns: +0 init must win
    peers[1][:8] = -0.0
    peers[2][:8] = -0.0
    peers[3][:8] = -0.0
    peers[0][8:12] = 3.4e38  # overflow to +inf inside the sum
    peers[1][8:12] = 3.4e38
    w = rng.choice(sp, size=64).astype(np.float32)
    w[:4] = -0.0
    return w, peers


def main():
    agg = import_reference()
    cases, small = [], {}

    def add_case(name, shapes, k, seed, store_full, w=None, peers=None):
        n = sum(int(np.prod(s)) for _, s in shapes)
        if peers is None:
            peers = [oracle.synth_np(n, seed, p, UPD_SCALE) for p in range(k)]
            w = oracle.synth_np(n, seed, W_PEER, W_SCALE)
        out = run_ref(agg, shapes, w, peers)
        # independent restatements must agree bit for bit with the reference
        w_np, _ = oracle.fedavg_np(peers, w)
        w_c, _ = oracle.fedavg(peers, w)
        same = lambda a, b: np.array_equal(a.view(np.uint32), b.view(np.uint32)) or \
            np.array_equal(np.isnan(a), np.isnan(b)) and np.array_equal(
                a[~np.isnan(a)].view(np.uint32), b[~np.isnan(b)].view(np.uint32))
        assert same(out, w_np), f"{name}: numpy restatement != reference"
        assert same(out, w_c), f"{name}: C restatement != reference"
        stride = max(1, n // 512)
        case = dict(name=name, shapes=[[nm, list(s)] for nm, s in shapes], k=k, seed=seed,
                    n=n, w_peer=W_PEER, upd_scale=UPD_SCALE, w_scale=W_SCALE, lr=0.1,
                    out_sha256=digest(out) if not np.isnan(out).any() else None,
                    sample_stride=stride,
                    sample_bits=[int(v) for v in out[::stride].view(np.uint32)])
        cases.append(case)
        if store_full:
            small[f"{name}__w"] = w
            small[f"{name}__out"] = out
            for i, p in enumerate(peers):
                small[f"{name}__peer{i}"] = p
        print(f"{name}: n={n} K={k} ok")

    add_case("mlp_k3", MLP_SHAPES, 3, 0x5EED0000, store_full=False)
    add_case("mlp_k7", MLP_SHAPES, 7, 0x5EED0007, store_full=False)
    add_case("odd_k1", [("a", (1,)), ("b", (7,)), ("c", (1001,))], 1, 0x5EED1001, True)
    add_case("odd_k7", [("a", (3, 5)), ("b", (1,)), ("c", (4099,))], 7, 0x5EED1007, True)
    add_case("flat_k2", [("a", (4096,))], 2, 0x5EED1002, True)
    add_case("flat_k64", [("a", (20011,))], 64, 0x5EED1064, False)
    add_case("flat_k256", [("a", (3001,))], 256, 0x5EED1256, False)
    w, peers = special_case()
    add_case("special_k4", [("a", (64,))], 4, 0, True, w=w, peers=peers)

    # ---- behaviour of the edge / error paths of the reference ----------
    behaviour = {}
    shapes = [("a", (5,))]
    model = Holder(shapes)
    before = model.state_dict()["a"].clone()
    node = types.SimpleNamespace(model=model, received_models=[], trainers_list=[],
                                 addr="127.0.0.1", port=1, neighbors=[])
    ret = agg.aggregate_models(node)  # reference :20-22
    behaviour["k0"] = dict(returns=repr(ret), model_unchanged=bool(torch.equal(before, model.state_dict()["a"])))

    model = Holder([("w", (4,)), ("nbt", ())], dtypes={"nbt": torch.int64})
    upd = {"w": torch.ones(4), "nbt": torch.tensor(3)}
    node = types.SimpleNamespace(model=model, received_models=[{"model": upd, "sender": 0}],
                                 trainers_list=[0], addr="127.0.0.1", port=1, neighbors=[])
    try:
        agg.aggregate_models(node)
        behaviour["int_buffer"] = dict(raises=None)
    except Exception as e:  # the reference raises at the true division (:32)
        behaviour["int_buffer"] = dict(raises=type(e).__name__, message=str(e),
                                       received_cleared=len(node.received_models) == 0)

    model = Holder([("a", (4,)), ("b", (2,))])
    node = types.SimpleNamespace(model=model, received_models=[{"model": {"a": torch.ones(4)}, "sender": 0}],
                                 trainers_list=[0], addr="127.0.0.1", port=1, neighbors=[])
    try:
        agg.aggregate_models(node)
        behaviour["missing_key"] = dict(raises=None)
    except Exception as e:
        behaviour["missing_key"] = dict(raises=type(e).__name__, message=str(e))

    # extra keys in an update are ignored (keys come from the model, :27)
    model = Holder([("a", (4,))])
    node = types.SimpleNamespace(model=model, received_models=[
        {"model": {"a": torch.ones(4), "zzz": torch.ones(9)}, "sender": 0}],
        trainers_list=[0], addr="127.0.0.1", port=1, neighbors=[])
    agg.aggregate_models(node)
    behaviour["extra_key"] = dict(result=[float(x) for x in model.state_dict()["a"]])

    meta = dict(generator="tests/golden/make_golden.py", reference="aggregator/aggregation.py:7-46",
                torch=torch.__version__, numpy=np.__version__, cases=cases, behaviour=behaviour)
    with open(os.path.join(HERE, "fedavg_golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    np.savez_compressed(os.path.join(HERE, "fedavg_small.npz"), **small)
    print(json.dumps(behaviour, indent=1))


if __name__ == "__main__":
    main()
