#!/usr/bin/env python3
"""Golden FedAvg vectors for float16 / bfloat16 models, from the REFERENCE's
own ``aggregate_models`` (reference aggregator/aggregation.py:7-46) run on
CPU here, through the same harness as make_golden.py (reference symlinked as
package ``p2pdl``, broadcast stubbed).  Build container only.

Inputs: the build's counter PRNG (``oracle.synth_np``) rounded to the
storage type; a special-value case (±0, subnormals, ±inf, NaN, overflow).
What is written (``fedavg16_golden.npz``): per case the storage bits of the
inputs and of the reference's result, and the case list as JSON.

Usage:  python tests/golden/make_golden_16.py   (from the repo root)
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import make_golden as MG  # noqa: E402  (the reference harness)
import oracle  # noqa: E402

DTYPES = {"float16": torch.float16, "bfloat16": torch.bfloat16}
CASES = [  # (name, K, shapes, seed)
    ("mlp_k3", 3, MG.MLP_SHAPES, 0x5EED1601),
    ("ragged_k7", 7, [("a", (3, 5)), ("b", (1,)), ("c", (1027,))], 0x5EED1602),
    ("k10", 10, [("x", (4099,))], 0x5EED1603),
]


def bits_of(t):
    return t.contiguous().view(torch.int16).numpy().view(np.uint16).reshape(-1)


def tensor_of(bits, dtype, shape):
    return torch.from_numpy(np.ascontiguousarray(bits, dtype=np.uint16).view(np.int16).copy()).view(
        DTYPES[dtype]).reshape(shape)


def run_ref(agg, shapes, dtype, w_bits, peer_bits):
    model = MG.Holder(shapes, dtypes={nm: DTYPES[dtype] for nm, _ in shapes})

    def split(bits):
        out, o = {}, 0
        for nm, s in shapes:
            n = int(np.prod(s))
            out[nm.replace(".", "__")] = tensor_of(bits[o:o + n], dtype, s)
            o += n
        return out

    with torch.no_grad():
        model.load_state_dict(split(w_bits))
    recv = [{"model": split(p), "sender": ("127.0.0.1", 7001 + i)} for i, p in enumerate(peer_bits)]
    node = types.SimpleNamespace(model=model, received_models=recv, trainers_list=[0] * len(recv),
                                 addr="127.0.0.1", port=7000, neighbors=[])
    agg.aggregate_models(node)
    return np.concatenate([bits_of(t.detach()) for t in model.state_dict().values()])


def special(dtype, k, n=96):
    rng = np.random.default_rng(1600 + k)
    sp = np.array([0.0, -0.0, 6e-8, -6e-8, 1e-5, 3e-5, np.inf, -np.inf, np.nan, 65504.0, -65504.0, 1.0,
                   -1.0, 0.1, 1 / 3, 1e-39, 3e38], dtype=np.float32)
    peers = [oracle.round_16(rng.choice(sp, size=n), dtype) for _ in range(k)]
    return oracle.round_16(rng.choice(sp, size=n), dtype), peers


def main():
    agg = MG.import_reference()
    meta, arrays = [], {}
    for dtype in DTYPES:
        todo = [(name, K, shapes, seed, None) for name, K, shapes, seed in CASES]
        todo.append(("special_k4", 4, [("a", (96,))], 0, special(dtype, 4)))
        for name, K, shapes, seed, given in todo:
            n = sum(int(np.prod(s)) for _, s in shapes)
            if given is None:
                w = oracle.round_16(oracle.synth_np(n, seed, MG.W_PEER, MG.W_SCALE), dtype)
                peers = [oracle.round_16(oracle.synth_np(n, seed, p, MG.UPD_SCALE), dtype) for p in range(K)]
            else:
                w, peers = given
            out = run_ref(agg, shapes, dtype, w, peers)

            def same(a, b):
                fa, fb = oracle.to_f32_16(a, dtype), oracle.to_f32_16(b, dtype)
                return bool(np.all((np.isnan(fa) & np.isnan(fb)) | (a == b)))

            agree = {mode: same(oracle.fedavg16_np(peers, w, dtype, torch_gpu=mode == "torch_gpu"), out)
                     for mode in ("true_div", "torch_gpu")}
            assert agree["true_div"], f"{dtype} {name}: the oracle's CPU mode != the reference"
            key = f"{dtype}__{name}"
            if n <= 20000:  # small cases in full; the MLP by digest (its inputs regenerate from the seed)
                arrays[f"{key}__w"] = w
                arrays[f"{key}__out"] = out
                for i, p in enumerate(peers):
                    arrays[f"{key}__peer{i}"] = p
            meta.append({"dtype": dtype, "name": name, "k": K, "shapes": [[nm, list(s)] for nm, s in shapes],
                         "seed": seed, "out_sha256": hashlib.sha256(out.tobytes()).hexdigest(),
                         "oracle_modes_equal_to_reference": agree})
            print(dtype, name, K, agree)
    arrays["meta"] = np.frombuffer(json.dumps({"generator": "tests/golden/make_golden_16.py",
                                               "reference": "aggregator/aggregation.py:7-46 (CPU)",
                                               "torch": torch.__version__, "cases": meta}).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "fedavg16_golden.npz"), **arrays)


if __name__ == "__main__":
    main()
