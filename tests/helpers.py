"""Shared test helpers (test infrastructure; may use the oracle)."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


def load_golden():
    with open(os.path.join(GOLDEN, "fedavg_golden.json")) as f:
        meta = json.load(f)
    small = np.load(os.path.join(GOLDEN, "fedavg_small.npz"))
    return meta, small


def case_inputs(case, small):
    """Regenerate (w, peers) flat float32 arrays of a golden case."""
    import oracle

    name, n, k = case["name"], case["n"], case["k"]
    if f"{name}__w" in small:
        return small[f"{name}__w"], [small[f"{name}__peer{i}"] for i in range(k)]
    w = oracle.synth(n, case["seed"], case["w_peer"], case["w_scale"])
    peers = [oracle.synth(n, case["seed"], p, case["upd_scale"]) for p in range(k)]
    return w, peers


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def assert_bits_equal(got, want, nan_equal=True, what=""):
    """Bit-exact float32 equality; NaNs compare equal as a class (payloads of
    NaNs produced by arithmetic are not specified across CPU/GPU)."""
    got = np.ascontiguousarray(got, dtype=np.float32)
    want = np.ascontiguousarray(want, dtype=np.float32)
    assert got.shape == want.shape, (got.shape, want.shape)
    if nan_equal:
        gn, wn = np.isnan(got), np.isnan(want)
        assert np.array_equal(gn, wn), f"{what}: NaN positions differ"
        got, want = got[~gn], want[~wn]
    bad = np.nonzero(bits(got) != bits(want))[0]
    assert bad.size == 0, (f"{what}: {bad.size} of {got.size} differ; first at {bad[0]}: "
                           f"got {got[bad[0]]!r} want {want[bad[0]]!r}")
