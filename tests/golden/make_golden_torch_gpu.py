#!/usr/bin/env python3
"""Golden FedAvg vectors for the reference AS DEPLOYED: its ops run by torch
on GPU tensors (the Node moves the model to cuda, reference
node/node.py:28-29, and unpickled updates are cuda tensors).

The reference cannot travel to the GPU box, so this script restates its
aggregation loop op for op in torch (reference aggregator/aggregation.py):
``acc = torch.zeros_like(param)`` (:15), ``acc += update[key]`` in
received_models order (:25-28), ``acc /= num_updates`` with the Python int K
(:31-32), and ``model.state_dict()[key] += learning_rate * acc`` with
``learning_rate = 0.1`` (:36-38) -- the same ATen calls on the same dtypes,
run on the GPU.  The differences from the CPU goldens (make_golden.py) are
ATen's: on a GPU tensor the division by the CPU scalar K is a multiply by
fl(1/K).

Run on a GPU box:  python tests/golden/make_golden_torch_gpu.py OUT.npz
What is written: per case the seed, K and shapes, the SHA-256 of the
updated model, and the full model for the small cases; inputs are
regenerated from the build's counter PRNG (``oracle.synth_np``).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle  # noqa: E402  (PRNG restatement only)

W_PEER = 0xFFFFF
UPD_SCALE, W_SCALE = 1e-2, 5e-2
MLP_SHAPES = [("fc1.weight", (512, 784)), ("fc1.bias", (512,)), ("fc2.weight", (256, 512)),
              ("fc2.bias", (256,)), ("fc3.weight", (10, 256)), ("fc3.bias", (10,))]
CASES = [  # (name, K, shapes, seed); full outputs stored below FULL_MAX elements
    ("mlp_k3", 3, MLP_SHAPES, 0x5EED1001),
    ("ragged_k7", 7, [("a", (3, 5)), ("b", (1,)), ("c", (1027,)), ("d", (2, 2, 3))], 0x5EED1002),
    ("k10", 10, [("x", (4099,)), ("y", (13,))], 0x5EED1003),
    ("k100", 100, [("x", (10007,))], 0x5EED1004),
    ("k256", 256, [("x", (2053,)), ("y", (6,))], 0x5EED1005),
]
FULL_MAX = 20000


def inputs(K, shapes, seed):
    n = sum(int(np.prod(s)) for _, s in shapes)
    return (oracle.synth_np(n, seed, W_PEER, W_SCALE),
            [oracle.synth_np(n, seed, p, UPD_SCALE) for p in range(K)])


def split(vec, shapes, dev):
    out, o = {}, 0
    for name, shape in shapes:
        k = int(np.prod(shape))
        out[name] = torch.from_numpy(vec[o:o + k].reshape(shape).copy()).to(dev)
        o += k
    return out


def reference_ops_on(dev, K, shapes, seed):
    """The reference's aggregation loop (aggregation.py:15-38) on `dev`."""
    w_flat, peer_flats = inputs(K, shapes, seed)
    state = split(w_flat, shapes, dev)
    received = [{"model": split(p, shapes, dev)} for p in peer_flats]
    acc = {key: torch.zeros_like(param) for key, param in state.items()}  # :15
    for rm in received:  # :25-28
        for key in acc:
            acc[key] += rm["model"][key]
    num_updates = len(received)
    for key in acc:  # :31-32
        acc[key] /= num_updates
    learning_rate = 0.1
    for key in state:  # :36-38
        state[key] += learning_rate * acc[key]
    return np.concatenate([t.cpu().numpy().reshape(-1) for t in state.values()])


def main(out_path):
    dev = torch.device("cuda", 0)
    meta, arrays = [], {}
    for name, K, shapes, seed in CASES:
        got = reference_ops_on(dev, K, shapes, seed)
        rec = {"name": name, "k": K, "shapes": [[nm, list(s)] for nm, s in shapes], "seed": seed,
               "sha256": hashlib.sha256(got.tobytes()).hexdigest(), "n": int(got.size)}
        if got.size <= FULL_MAX:
            arrays[name] = got
        meta.append(rec)
    arrays["meta"] = np.frombuffer(json.dumps({"device": torch.cuda.get_device_name(0), "torch": torch.__version__,
                                               "cases": meta}).encode(), dtype=np.uint8)
    np.savez_compressed(out_path, **arrays)
    print(json.dumps(meta, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "fedavg_torch_gpu.npz"))
