"""The padded robust kernels' layout (robust.hip PAD, robust_pair.hip PAD):
K real keys in a KP-slot network, `lo` pads at the bottom of the order and
the rest at the top, the network's fixed ranks then hold the answer.  This
restates the pad arithmetic and the fit conditions in numpy and checks them
against the oracle's rules on every K they cover (ties and +-inf included);
the GPU tests check the kernels themselves."""
import numpy as np
import pytest

import oracle


def pad_lo(KP, rule, K, b):  # robust.hip pad_lo; robust_pair.hip pair_tile (KP = 256)
    return (KP - 1) // 2 - (K - 1) // 2 if rule == "median" else (KP * 2) // 10 - b


def fits(KP, rule, K, b):  # robust.hip robust_pad_fits; robust_pair.hip p2p_robust_pair_fits
    if K > KP or 2 * K <= KP:
        return False
    if rule == "median":
        return True
    b0 = (KP * 2) // 10
    return 0 <= b <= b0 and K - b <= KP - b0 and 1 <= K - 2 * b <= KP - 2 * b0


def padded_answer(x, KP, rule, b):
    """What the fixed network reads from the padded, sorted slots."""
    K = x.size
    lo = pad_lo(KP, rule, K, b)
    slots = np.concatenate([x, np.full(lo, -np.inf, np.float32), np.full(KP - K - lo, np.inf, np.float32)])
    s = slots[np.argsort(oracle.f2key_np(slots), kind="stable")]  # the total order: -0 < +0
    if rule == "median":
        return s[(KP - 1) // 2]
    b0 = (KP * 2) // 10
    acc = np.float32(0)
    with np.errstate(invalid="ignore"):  # +inf and -inf both kept: NaN, as the oracle
        for v in s[b0:b0 + K - 2 * b]:  # ascending sum of the kept ranks
            acc = np.float32(acc + v)
    return np.float32(acc / np.float32(K - 2 * b))


@pytest.mark.parametrize("KP", [64, 128, 256])
def test_default_trim_always_fits(KP):
    for K in range(KP // 2 + 1, KP + 1):
        assert fits(KP, "median", K, 0)
        assert fits(KP, "trimmed", K, oracle.trim_count(K)), K


@pytest.mark.parametrize("KP", [64, 128, 256])
@pytest.mark.parametrize("rule", ["median", "trimmed"])
def test_padded_ranks_give_the_rule(KP, rule):
    rng = np.random.default_rng(KP)
    for K in range(KP // 2 + 1, KP + 1):
        bs = [oracle.trim_count(K)] if rule == "median" else sorted({oracle.trim_count(K), 0, K // 4, K // 2 - 1})
        for b in bs:
            if not fits(KP, rule, K, b):
                continue
            for trial in range(3):
                x = np.round(rng.standard_normal(K) * 4).astype(np.float32)  # ties
                if trial == 1:
                    x[rng.integers(0, K, 3)] = np.inf
                    x[rng.integers(0, K, 3)] = -np.inf
                got = padded_answer(x, KP, rule, b)
                _, want = oracle.robust([np.array([v], np.float32) for v in x], 1 if rule == "median" else 2,
                                        b if rule == "trimmed" else 0)
                assert np.array_equal(np.array([got], np.float32).view(np.uint32), want.view(np.uint32)) or \
                    (np.isnan(got) and np.isnan(want[0])), (KP, rule, K, b, got, want)


def test_fit_boundaries():
    # pair kernel (KP = 256): b <= 51, K - b <= 205, K - 2b <= 154
    assert fits(256, "trimmed", 200, 40) and not fits(256, "trimmed", 200, 10) and not fits(256, "trimmed", 256, 40)
    assert fits(256, "trimmed", 129, 0) and fits(256, "trimmed", 150, 51) and not fits(256, "trimmed", 150, 52)
    # K <= 128 kernels
    assert fits(128, "trimmed", 100, 15) and not fits(128, "trimmed", 100, 10) and fits(128, "trimmed", 65, 0)
    assert not fits(128, "median", 64, 0)  # K <= KP / 2 runs the KP = 64 kernels
