"""The oracle itself, pinned against the reference's golden vectors and KATs (CPU)."""
import hashlib
import os
import sys

import numpy as np
import pytest
import torch

import oracle
from helpers import assert_bits_equal, case_inputs, load_golden

META, SMALL = load_golden()


@pytest.mark.parametrize("case", META["cases"], ids=lambda c: c["name"])
def test_c_and_numpy_oracles_match_reference_golden(case):
    w, peers = case_inputs(case, SMALL)
    for fn in (oracle.fedavg, oracle.fedavg_np):
        out, _ = fn(peers, w, lr=case["lr"])
        stride = case["sample_stride"]
        want = np.array(case["sample_bits"], dtype=np.uint32).view(np.float32)
        assert_bits_equal(out[::stride], want, what=f"{fn.__name__} {case['name']}")
        if case["out_sha256"]:
            assert hashlib.sha256(out.tobytes()).hexdigest() == case["out_sha256"]
        if f"{case['name']}__out" in SMALL:
            assert_bits_equal(out, SMALL[f"{case['name']}__out"])


def test_golden_inputs_regenerate_from_numpy_prng():
    """The golden inputs were made with oracle.synth_np; the C PRNG agrees."""
    for case in META["cases"]:
        if case["name"] == "special_k4":
            continue
        n = min(case["n"], 5000)
        a = oracle.synth(n, case["seed"], 1, case["upd_scale"])
        b = oracle.synth_np(n, case["seed"], 1, case["upd_scale"])
        assert_bits_equal(a, b)


def test_reference_error_behaviour_recorded():
    b = META["behaviour"]
    assert b["k0"] == {"returns": "None", "model_unchanged": True}
    assert b["int_buffer"]["raises"] == "RuntimeError"
    assert b["missing_key"]["raises"] == "KeyError"


def test_sha256_kats_and_hashlib():
    kats = {b"": "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855",
            b"abc": "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad",
            b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq":
                "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1",
            b"a" * 1_000_000: "cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0"}
    for m, h in kats.items():
        assert oracle.sha256(m).hex() == h
    rng = np.random.default_rng(0)
    for L in [1, 55, 56, 63, 64, 65, 119, 120, 128, 1000, 70001]:
        m = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        assert oracle.sha256(m) == hashlib.sha256(m).digest()


@pytest.mark.parametrize("k", [1, 2, 3, 8, 33, 128, 256])
def test_robust_oracles_agree(k):
    n = 2000
    peers = [oracle.synth(n, k, p, 1.0) for p in range(k)]
    peers[0][:50] = np.nan
    peers[-1][50:100] = -0.0
    for rule, b in [(1, 0), (2, oracle.trim_count(k))]:
        _, c = oracle.robust(peers, rule, b)
        npv = oracle.robust_np(peers, rule, b)
        assert_bits_equal(c, npv, nan_equal=(rule == 2), what=f"rule {rule} K={k}")


def test_median_matches_torch_median_nan_free():
    x = torch.randn(64, 5000, generator=torch.Generator().manual_seed(1))
    x[:, :10] = 0.0
    _, c = oracle.robust(list(x.numpy()), 1)
    assert np.array_equal(c, x.median(dim=0).values.numpy())


def test_trim_count():
    assert [oracle.trim_count(k) for k in (1, 2, 4, 5, 9, 10, 128, 256)] == [0, 0, 0, 1, 1, 2, 25, 51]


def test_sorting_networks_0_1_principle():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "p2pdl_amd", "csrc"))
    import gen_networks

    gen_networks.check()


def test_committed_networks_are_the_generated_ones():
    """networks.inc (what the kernels compile) is exactly gen_networks.py's
    checked output, three-input lowering included."""
    csrc = os.path.join(os.path.dirname(os.path.dirname(__file__)), "p2pdl_amd", "csrc")
    sys.path.insert(0, csrc)
    import gen_networks

    with open(os.path.join(csrc, "networks.inc")) as f:
        assert f.read() == "\n".join(gen_networks.emit_fused())


def test_three_list_merges_close_with_one_operation_per_output():
    """The three-list merge (gen_networks.MSort): every output of a merge of
    three sorted lists is one min / max / min3 / max3 / med3, proved on the
    stage's 0-1 domain as it is built and re-checked here on random sorted
    lists of integers with ties; four lists do not close that way."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "p2pdl_amd", "csrc"))
    import gen_networks as G

    rng = np.random.default_rng(3)
    for sizes in [(3, 3, 2), (8, 8, 8), (9, 6, 6), (15, 14, 14)]:
        n = sum(sizes)
        net = G.MSort(n)
        lists, i = [], 0
        for s in sizes:
            lists.append(list(range(i, i + s)))
            i += s
        outs = net.merge(lists)
        prog = G.MSortProgram(n, range(n), net=(net, outs)).fuse()
        x = rng.integers(0, 5, size=(500, n)).astype(np.uint64)
        i = 0
        for s in sizes:
            x[:, i:i + s] = np.sort(x[:, i:i + s], axis=1)
            i += s
        assert np.array_equal(prog.run(x), np.sort(x, axis=1)), sizes
    assert G.merge_cost((8, 8, 8)) == 82  # two lowered Batcher merges: 37 + 60
    with pytest.raises(AssertionError):
        G.MSort(16).merge([[0, 1, 2, 3], [4, 5, 6, 7], [8, 9, 10, 11], [12, 13, 14, 15]])


def test_delta_snapshot_oracle_matches_torch_reference_ops():
    """oracle.delta_snapshot_np == the reference's torch ops (node/node.py:275,279,282)."""
    import torch

    cur = oracle.synth(10_001, 3, 1, 1e-1)
    prev = oracle.synth(10_001, 3, 2, 1e-1)
    d, p = oracle.delta_snapshot_np(cur, prev)
    assert np.array_equal(d.view(np.uint32), (torch.from_numpy(cur) - torch.from_numpy(prev)).numpy().view(np.uint32))
    assert np.array_equal(p, cur)
    d0, p0 = oracle.delta_snapshot_np(cur, None)
    assert np.array_equal(d0, cur) and np.array_equal(p0, cur) and d0 is not cur


def test_synth_at_matches_synth():
    idx = np.array([0, 1, 17, 4095, 99_999])
    full = oracle.synth(100_000, 0x5EED0001, 3, 1e-2)
    assert np.array_equal(oracle.synth_at(idx, 0x5EED0001, 3, 1e-2), full[idx])


@pytest.mark.parametrize("k", [5, 10, 128, 256])
def test_trimmed_mean_oracle_pinned_to_scipy_bit_exact(k):
    """External pin of the build-defined trimmed mean:
    scipy.stats.trim_mean(x, 0.2, axis=0) cuts int(0.2 K) per end, as
    trim_count does.  With integer-valued fp32 inputs every partial sum is
    exact (|sum| < 2**24), so summation order cannot matter and the fp32
    quotients must agree bit for bit."""
    from scipy import stats

    n = 20_000
    rng = np.random.default_rng(k)
    x = rng.integers(-1000, 1001, size=(k, n)).astype(np.float32)
    x[:, :500] = rng.integers(-3, 4, size=(k, 500))  # heavy ties
    b = oracle.trim_count(k)
    assert b == int(0.2 * k)
    _, got = oracle.robust(list(x), oracle.RULE_TRIMMED, b)
    want = stats.trim_mean(x, 0.2, axis=0)
    assert want.dtype == np.float32
    assert_bits_equal(got, want, what=f"trim_mean K={k}")
    assert_bits_equal(oracle.robust_np(list(x), oracle.RULE_TRIMMED, b), want, what=f"numpy K={k}")


@pytest.mark.parametrize("k", [5, 10, 128, 255, 256])
def test_median_oracle_pinned_to_torch_median_integer_ties(k):
    """torch.median (lower median for even K) on integer-valued data with
    many ties, both signs (NaN-free: torch propagates NaN, the key order ranks
    it)."""
    n = 20_000
    rng = np.random.default_rng(100 + k)
    x = rng.integers(-50, 51, size=(k, n)).astype(np.float32)
    _, got = oracle.robust(list(x), oracle.RULE_MEDIAN)
    want = torch.from_numpy(x).median(dim=0).values.numpy()
    assert_bits_equal(got, want, nan_equal=False, what=f"median K={k}")
