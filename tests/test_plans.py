"""CPU checks of the host-side launch plans of the FedAvg split kernel
(p2pdl_amd/ops.py): the chunk list of a state_dict of separately allocated
tensors (include/p2pdl.h p2p_fedavg_split_chunks_f32) and the route switch.
No GPU: the library's plan helper reads the CU count from the device when
there is one and falls back to 256 otherwise; the pointers are synthetic."""
import numpy as np
import pytest

from p2pdl_amd import _native as N
from p2pdl_amd import ops

CUS = 256  # p2p_fedavg_split_plan's fallback without a device


def _ptrs(L, K, base=1 << 30):
    return (np.arange(L * K, dtype=np.uint64).reshape(L, K) * np.uint64(1 << 22)) + np.uint64(base)


def test_chunk_plan_layout():
    if int(N.lib().p2p_fedavg_split_plan(16, CUS)) != CUS:
        pytest.skip("a device with another CU count is visible")
    n = np.array([1_234_567, 3, 0, 8 * 1024 * CUS], dtype=np.int64)
    ptrs = _ptrs(4, 16)
    mask, lst = ops._chunk_plan(ptrs, [1 << 24] * 4, None, n, 16, 0)
    assert list(mask) == [True, True, False, True]  # an empty key takes no chunk
    nch = [-(-int(m) // 1024) if m else 0 for m in n]
    C = sum(nch)
    assert len(lst) == 8 * -(-C // 8) and lst.dtype == ops._SPLIT_DTYPE
    assert (lst["seg"][:nch[0]] == 0).all() and (lst["c0"][:nch[0]] == np.arange(nch[0]) * 1024).all()
    assert lst["seg"][nch[0]] == 1 and lst["c0"][nch[0]] == 0
    assert (lst["seg"][nch[0] + 1:C] == 3).all() and (lst["seg"][C:] == -1).all() and (lst["c0"][C:] == 0).all()


def test_chunk_plan_declines():
    n = np.array([8 * 1024 * CUS], dtype=np.int64)
    ptrs = _ptrs(1, 16)
    assert ops._chunk_plan(ptrs, [1 << 24], None, n, 15, 0) is None            # K < 16
    assert ops._chunk_plan(ptrs, [1 << 24], None, n, 16, ops.P2P_RULE_MEDIAN) is None  # a robust rule
    assert ops._chunk_plan(ptrs, [1 << 24], None, np.array([1024 * 100]), 16, 0) is None  # under a CU round
    odd = ptrs.copy()
    odd[0, 5] += np.uint64(4)  # one peer view 4-B aligned only: no chunked key left
    assert ops._chunk_plan(odd, [1 << 24], None, n, 16, 0) is None
    assert ops._chunk_plan(ptrs, [(1 << 24) + 8], None, n, 16, 0) is None      # w 8-B aligned
    assert ops._chunk_plan(ptrs, [1 << 24], [(1 << 24) + 4], n, 16, 0) is None  # out 4-B aligned


def test_state_dict_route_is_checked():
    assert ops.STATE_DICT_ROUTE == "chunks"  # the product route


@pytest.mark.parametrize("K,route", [(3, "chunks"), (64, "chunks"), (64, "tiles"), (64, "vgpr"), (20, "chunks")])
def test_layout_cache_writes_the_same_table(monkeypatch, K, route):
    """A segment-table launch whose layout is cached (ops._LAYOUTS: same
    element counts, K, rule and alignment, new addresses) produces the very
    bytes a cold build produces for those addresses -- the device image and
    the launch entry -- with a misaligned key and ragged sizes in the mix.
    The device side is faked (no GPU): the image handed to the H2D copy and
    the entry handed to the launch are captured."""
    import torch

    sizes = [1_234_567, 5, 0, 300_001, 2_000_000, 17]
    L = len(sizes)
    seen = {}

    class FakeBuf:
        def __init__(self, n):
            self.n = n

        def data_ptr(self):
            return 1 << 33

    real_empty = torch.empty

    def fake_empty(*a, **k):
        if str(k.get("device", "")).startswith("cuda"):
            return FakeBuf(a[0])
        return real_empty(*a, **k)

    class FakeStream:
        cuda_stream = 0

    monkeypatch.setattr(ops.torch, "empty", fake_empty)
    monkeypatch.setattr(ops._RING, "to_device", lambda host, dev, out=None: seen.__setitem__("host", host.copy()))
    monkeypatch.setattr(ops, "_launch_entry", lambda entry, *a: seen.__setitem__("entry", entry[1:4] + entry[5:]))
    monkeypatch.setattr(ops.torch.cuda, "current_stream", lambda dev=None: FakeStream())
    monkeypatch.setattr(ops.torch.cuda, "device", lambda d: __import__("contextlib").nullcontext())
    monkeypatch.setattr(ops.N, "stream_handle", lambda *a: 0)
    monkeypatch.setattr(ops, "STATE_DICT_ROUTE", route)
    monkeypatch.setattr(ops, "SPLIT_SEGMENT_MIN_TILES", 0)
    dev = torch.device("cuda", 0)
    ws = [real_empty(max(n, 1)) for n in sizes]

    def run(ptrs):
        seen.clear()
        ops._launch_segments(ws, ptrs, sizes, "fedavg", K, 0.1, None, 0.2, None, dev)
        return seen.get("host"), seen.get("entry")

    a = _ptrs(L, K)
    a[3, 1] += np.uint64(4)  # key 3: one peer view 4-B aligned only
    b = a + np.uint64(1 << 40)  # new addresses, the same alignment
    ops._LAYOUTS.clear()
    run(a)
    warm_host, warm_entry = run(b)  # layout from a's build
    ops._LAYOUTS.clear()
    cold_host, cold_entry = run(b)
    assert warm_host is not None and np.array_equal(warm_host, cold_host)
    assert warm_entry == cold_entry
