"""The broadcast envelope (p2pdl_amd.node.envelope):
its storage blobs are byte-identical to torch's legacy storage pickling, and
the envelope loads with pickle.loads (reference node/node.py:112) and with
the product's restricted parser exactly like the reference's
pickle.dumps({"type": "global_model_update", "model": state_dict, ...})
(reference aggregator/aggregation.py:70)."""
import collections
import io
import pickle
import warnings

import numpy as np
import pytest
import torch

from p2pdl_amd.node import envelope as E
from p2pdl_amd.node.inbox import ZeroCopyParser


def _torch_blob(t):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        fn, (blob,) = t.storage().__reduce__()
    assert fn is torch.storage._load_from_bytes
    return blob


@pytest.mark.parametrize("n", [0, 1, 6, 255, 256, 65_536, 100_003])
def test_blob_header_is_torchs(n):
    t = torch.arange(n, dtype=torch.float32)
    blob = _torch_blob(t)
    f = io.BytesIO(blob)
    for _ in range(3):
        pickle.Unpickler(f).load()
    keys = []

    class U(pickle.Unpickler):
        def persistent_load(self, pid):
            keys.append(pid[2])

    U(f).load()
    assert E.legacy_storage_header(n, keys[0]) + t.numpy().tobytes() == blob


def _blob_key_location(blob):
    f = io.BytesIO(blob)
    for _ in range(3):
        pickle.Unpickler(f).load()
    pids = []

    class U(pickle.Unpickler):
        def persistent_load(self, pid):
            pids.append(pid)

    U(f).load()
    return pids[0][2], pids[0][3]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 255, 100_003])
def test_blob_header_is_torchs_on_the_gpu(cuda, n):
    """A CUDA storage's blob names its location ('cuda:0'), as torch's
    pickle of the reference's GPU state_dict does."""
    t = torch.arange(n, dtype=torch.float32, device=cuda)
    blob = _torch_blob(t)
    key, loc = _blob_key_location(blob)
    assert loc == torch.serialization.location_tag(t.untyped_storage()) and loc.startswith("cuda:")
    assert E.legacy_storage_header(n, key, loc) + t.cpu().numpy().tobytes() == blob


def _state():
    return collections.OrderedDict([
        ("fc.weight", torch.randn(33, 17)), ("fc.bias", torch.randn(33)),
        ("bn.running_mean", torch.zeros(33)), ("bn.num_batches_tracked", torch.tensor(7)),
        ("empty", torch.zeros(0)), ("strided", torch.randn(5, 3).t()), ("half", torch.randn(4).half()),
    ])


def test_envelope_loads_like_the_reference():
    sd = _state()
    ours = E.global_model_envelope(sd, "10.0.0.1", 5001)
    ref = pickle.dumps({"type": "global_model_update", "model": sd, "addr": "10.0.0.1", "port": 5001})
    a, b = pickle.loads(ours), pickle.loads(ref)
    assert {k: v for k, v in a.items() if k != "model"} == {k: v for k, v in b.items() if k != "model"}
    assert type(a["model"]) is collections.OrderedDict and list(a["model"]) == list(sd)
    for k, v in sd.items():
        got = a["model"][k]
        assert got.dtype == v.dtype and got.shape == v.shape and got.stride() == v.stride(), k
        assert torch.equal(got, v), k
        assert got.untyped_storage().nbytes() == v.untyped_storage().nbytes(), k


def test_envelope_parts_alias_the_slots_and_join_to_the_envelope():
    sd = _state()
    sd["big"] = torch.randn(200, 200)  # above the pickler's 64 KiB frame: handed over, not framed
    with E.LOCK:
        parts = E.envelope_parts(sd, "h", 1)
        big = [p for p in parts if p.nbytes >= 200 * 200 * 4]
        assert len(big) == 1 and not isinstance(big[0].obj, bytes)  # a view of the slot, not a copy
        joined = b"".join(parts)
    assert pickle.loads(joined)["model"].keys() == sd.keys()
    assert joined == E.global_model_envelope(sd, "h", 1)


def test_pickler_hands_large_blobs_over_uncopied():
    """envelope._fill waits only for the DMAs of blobs below _INLINE_MAX
    before pickling: CPython's pickler copies smaller in-band payloads into
    its frame (it reads them then) and hands larger ones to the writer as
    the object itself (read only when the parts are).  Pin both halves: a
    blob of _INLINE_MAX bytes written after pickling shows in the parts, and
    the pickler's own cut-off lies below _INLINE_MAX."""
    def aliased(size):
        buf = bytearray(size)
        out = E._Parts()
        pickle.Pickler(out, protocol=5).dump({"blob": E._Blob(memoryview(buf).toreadonly())})
        buf[:4] = b"late"  # the DMA landing after the pickler ran
        return b"late" in b"".join(out.parts)

    assert aliased(E._INLINE_MAX) and not aliased(1024)
    cut = next(s for s in (1 << k for k in range(10, 21)) if aliased(s))
    assert cut <= E._INLINE_MAX // 4, cut  # 64 KiB on CPython 3.8-3.13


def test_envelope_passes_the_restricted_parser():
    """A peer running p2pdl_amd's receive path parses the global model with
    the restricted machine (no unpickler on peer bytes): same payloads."""
    sd = collections.OrderedDict((k, v) for k, v in _state().items() if k not in ("bn.num_batches_tracked",))
    with E.LOCK:  # the model as the envelope encodes it (protocol 5, in-band blobs)
        blob = pickle.dumps(E._placeholders(sd), protocol=5)
    raw = ZeroCopyParser(blob).parse()
    for k, v in sd.items():
        arr = np.ascontiguousarray(raw[k].array()).reshape(-1)
        assert np.array_equal(arr.view(np.uint8), v.contiguous().numpy().reshape(-1).view(np.uint8)), k


def test_dumps_state_is_a_state_dict_pickle():
    """The trainer's update (reference node/node.py:285) by the same route:
    pickle.loads and the restricted parser read the state back; the global
    model's layout is left alone."""
    sd = _state()
    g = E.global_model_envelope(sd, "h", 1)
    upd = collections.OrderedDict((k, v * 2) for k, v in sd.items() if v.dtype == torch.float32)
    data = E.dumps_state(upd)
    back = pickle.loads(data)
    assert type(back) is collections.OrderedDict and list(back) == list(upd)
    assert all(torch.equal(back[k], v) for k, v in upd.items())
    raw = ZeroCopyParser(data).parse()
    for k, v in upd.items():
        arr = np.ascontiguousarray(raw[k].array()).reshape(-1)
        assert np.array_equal(arr.view(np.uint8), v.contiguous().numpy().reshape(-1).view(np.uint8)), k
    assert E.global_model_envelope(sd, "h", 1) == g  # its own layout, untouched


@pytest.mark.gpu
def test_envelope_from_gpu_model(cuda):
    net = torch.nn.Sequential(torch.nn.Linear(33, 64), torch.nn.BatchNorm1d(64), torch.nn.Linear(64, 10)).to(cuda)
    sd = net.state_dict()
    for _ in range(2):  # the second call reuses the pinned layout
        got = pickle.loads(E.global_model_envelope(sd, "a", 2))["model"]
        upd = pickle.loads(E.dumps_state(sd))  # the trainer's route, its own layout
        assert list(got) == list(sd) and list(upd) == list(sd)
        ref = pickle.loads(pickle.dumps({"model": sd}))["model"]  # the reference's envelope
        for k, v in sd.items():
            assert got[k].device == ref[k].device == v.device and upd[k].device == v.device, k
            assert torch.equal(got[k], v) and torch.equal(upd[k], v), k
        with torch.no_grad():
            for p in net.parameters():
                p.add_(1.0)  # new values, same layout


@pytest.mark.gpu
def test_envelope_large_gpu_tensors_settle_before_the_parts_are_read(cuda):
    """Blobs of _INLINE_MAX bytes or more are DMA'd while the pickler runs
    (envelope._fill) and waited for before the parts are handed out: every
    call's envelope and update carry the values of that call, bit for bit,
    with each round's new values written by a kernel just before it."""
    sd = collections.OrderedDict([("conv.weight", torch.empty(512, 512, 3, 3, device=cuda)),
                                  ("bn.weight", torch.empty(512, device=cuda)),
                                  ("fc.weight", torch.empty(1000, 512, device=cuda)),
                                  ("small", torch.empty(70_000, device=cuda))])
    for rnd in range(3):
        with torch.no_grad():
            for i, t in enumerate(sd.values()):
                t.copy_(torch.arange(t.numel(), device=cuda, dtype=torch.float32).view_as(t) * (rnd + 1) + i)
        with E.LOCK:
            joined = b"".join(E.envelope_parts(sd, "h", 1))
        got = pickle.loads(joined)["model"]
        upd = pickle.loads(E.dumps_state(sd))
        for k, v in sd.items():
            assert torch.equal(got[k], v) and torch.equal(upd[k], v), (rnd, k)


@pytest.mark.gpu
@pytest.mark.parametrize("image_max", [0, 1 << 30])
def test_envelope_device_image_only_below_the_cap(cuda, monkeypatch, image_max):
    """a layout's device image stays resident, so models above
    DEVICE_IMAGE_MAX take per-tensor DMAs (no image); both routes give the
    reference's bytes."""
    monkeypatch.setattr(E, "DEVICE_IMAGE_MAX", image_max)
    monkeypatch.setattr(E, "_LAYOUTS", {})
    net = torch.nn.Sequential(torch.nn.Linear(33, 64), torch.nn.BatchNorm1d(64), torch.nn.Linear(64, 10)).to(cuda)
    sd = net.state_dict()
    got = pickle.loads(E.global_model_envelope(sd, "a", 2))["model"]
    (lay,) = E._LAYOUTS.values()
    assert (lay.dev is None) == (image_max == 0)
    for k, v in sd.items():
        assert got[k].device == v.device and torch.equal(got[k], v), k
