"""The global model's broadcast envelope, serialized with one copy of the
weights (reference aggregator/aggregation.py:66-70).

The reference pickles ``{"type": "global_model_update", "model":
state_dict, "addr", "port"}`` with the CUDA tensors inside.  torch pickles a
tensor as ``torch._utils._rebuild_tensor_v2(storage, offset, size, stride,
requires_grad, OrderedDict())`` and each storage as
``torch.storage._load_from_bytes(blob)``, the blob being torch's legacy
``torch.save`` stream of that storage: four small pickles (magic number,
protocol version 1001, sys_info, a persistent-id reference), the storage key
list, an 8-byte element count and the raw bytes.  Building it, torch copies
each storage to the host, into a BytesIO, out of it, and into the pickle:
three copies of every weight after the device-to-host one.

Here the fp32 weights land by device-to-host DMA straight into a pinned
buffer laid out as those blobs -- each blob's header and count written once
when the buffer is made (they depend on the tensor sizes only) -- and the
envelope is pickled with protocol 5, each blob an in-band ``PickleBuffer``
over its slot, which the pickler hands to its writer uncopied: the
broadcast sends the weights straight from the DMA target
(``envelope_parts``), or one join makes the bytes (``global_model_envelope``).  The
receiver's ``pickle.loads`` (reference node/node.py:112) and
``p2pdl_amd.node.inbox.ZeroCopyParser`` read it like torch's own pickle
(``tests/test_envelope.py`` checks the blobs against ``torch.save`` byte for
byte and the envelope against ``pickle.loads``).  Each blob names its
storage's own location, as torch's does ('cuda:0' for the reference's GPU
model), so ``pickle.loads`` puts every tensor on the device the reference's
envelope puts it on.
"""
from __future__ import annotations

import collections
import io
import pickle
import threading

import numpy as np
import torch

__all__ = ["LOCK", "dumps_state", "envelope_parts", "global_model_envelope", "legacy_storage_header"]

# torch.serialization's legacy stream: magic number, protocol version, sys_info
_MAGIC = 0x1950A86A20F9469CFC6C
_PROTOCOL_VERSION = 1001
_SYS_INFO = {"protocol_version": _PROTOCOL_VERSION, "little_endian": True,
             "type_sizes": {"short": 2, "int": 4, "long": 4}}


class _StorageRef:
    """Stands for the storage in the header's persistent-id pickle."""


def legacy_storage_header(numel: int, key: str, location: str = "cpu") -> bytes:
    """The bytes torch's legacy ``torch.save`` of a float32 storage of
    ``numel`` elements on ``location`` ('cpu', 'cuda:0', ...) writes before
    the raw data: the four header pickles (protocol 2, as torch writes them),
    the key list and the 8-byte count."""
    f = io.BytesIO()
    pickle.dump(_MAGIC, f, protocol=2)
    pickle.dump(_PROTOCOL_VERSION, f, protocol=2)
    pickle.dump(_SYS_INFO, f, protocol=2)
    ref = _StorageRef()

    class _P(pickle.Pickler):
        def persistent_id(self, obj):
            if obj is ref:
                return ("storage", torch.FloatStorage, key, location, numel, None)
            return None

    _P(f, protocol=2).dump(ref)
    pickle.dump([key], f, protocol=2)
    f.write(int(numel).to_bytes(8, "little"))
    return f.getvalue()


class _Blob:
    """Pickles as torch.storage._load_from_bytes(<the slot's bytes>)."""
    __slots__ = ("mv",)

    def __init__(self, mv):
        self.mv = mv

    def __reduce__(self):
        return (torch.storage._load_from_bytes, (pickle.PickleBuffer(self.mv),))


class _Tensor:
    """Pickles as torch._utils._rebuild_tensor_v2 over a _Blob, as torch
    pickles a contiguous CPU tensor."""
    __slots__ = ("blob", "size", "stride")

    def __init__(self, blob, size, stride):
        self.blob, self.size, self.stride = blob, size, stride

    def __reduce__(self):
        return (torch._utils._rebuild_tensor_v2,
                (self.blob, 0, self.size, self.stride, False, collections.OrderedDict()))


class _Layout:
    """One pinned buffer of legacy blobs for a fixed list of fp32 sizes and
    storage locations.  The blobs the pickler copies (below _INLINE_MAX)
    come first, then the large ones; every payload starts 256-B aligned
    (the slots are separate views, so the gaps never reach the pickle).
    For a model on one GPU a device image of the buffer (headers written
    once) takes the weights by one gather kernel, and two DMAs bring it
    over: the small blobs' region, then the rest."""

    def __init__(self, numels, locations, pin: bool, device=None):
        heads = [legacy_storage_header(n, str(i), loc) for i, (n, loc) in enumerate(zip(numels, locations))]
        order = sorted(range(len(heads)), key=lambda i: len(heads[i]) + 4 * numels[i] >= _INLINE_MAX)
        self.spans = [None] * len(heads)  # (blob start, payload start, blob end) per tensor
        off = self.inline_end = 0
        for i in order:
            a = -(-(off + len(heads[i])) // 256) * 256 - len(heads[i])
            self.spans[i] = (a, a + len(heads[i]), a + len(heads[i]) + 4 * numels[i])
            off = self.spans[i][2]
            if len(heads[i]) + 4 * numels[i] < _INLINE_MAX:
                self.inline_end = off
        self.buf = torch.empty(max(off, 1), dtype=torch.uint8, pin_memory=pin)  # DMA target for GPU weights
        arr = self.buf.numpy()
        arr[:] = 0
        for h, (a, p, _) in zip(heads, self.spans):
            arr[a:p] = np.frombuffer(h, dtype=np.uint8)
        self.mv = memoryview(arr).toreadonly()
        self.dev = None
        if device is not None:
            self.dev = torch.empty_like(self.buf, device=device)
            self.dev.copy_(self.buf)  # the headers, once
            torch.cuda.current_stream(device).synchronize()
        self.gather = None  # (source pointers, device table, base, span, segments, tiles)


_LAYOUTS = {}
# Largest model (fp32 bytes) given a device image: each layout keeps one for
# the life of the process, so at most two (the 'global' and 'update'
# purposes) of this size stay on the GPU.  The cfg2 ResNet-18
# (47 MB) and every model below it take the gather kernel; a larger model
# (cfg3's 4 GB) takes per-tensor DMAs from its own memory.
DEVICE_IMAGE_MAX = 1 << 30
LOCK = threading.RLock()  # held while envelope parts (which alias the pinned buffer) are in use


class _Parts:
    """The pickler's output as the buffers it hands over: small frames as
    bytes, each weight blob as a view of its pinned slot (no copy)."""

    def __init__(self):
        self.parts = []
        self.nbytes = 0

    def write(self, b):
        m = memoryview(b)
        self.parts.append(m)
        self.nbytes += m.nbytes
        return m.nbytes


def _layout_for(purpose, fast):
    locs = tuple(torch.serialization.location_tag(t.untyped_storage()) for _, t in fast)
    sig = (purpose, locs, tuple(t.numel() for _, t in fast))
    lay = _LAYOUTS.get(sig)
    if lay is None:
        devs = {t.device for _, t in fast}
        one_gpu = len(devs) == 1 and next(iter(devs)).type == "cuda"
        # the device image stays resident with its layout (one per purpose):
        # above DEVICE_IMAGE_MAX the tensors take one DMA each instead
        one_gpu = one_gpu and sum(4 * t.numel() for _, t in fast) <= DEVICE_IMAGE_MAX
        lay = _Layout(sig[2], locs, any(t.is_cuda for _, t in fast), next(iter(devs)) if one_gpu else None)
        for old in [k for k in _LAYOUTS if k[0] == purpose]:
            del _LAYOUTS[old]  # one model per purpose: keep the latest layout only
        _LAYOUTS[sig] = lay
    return lay


# A blob below this size is copied into the pickler's frame while it
# pickles (CPython's _pickle hands a payload of FRAME_SIZE_TARGET = 64 KiB or
# more to the writer as the object itself, uncopied): its DMA must have
# landed before the pickler runs, a larger one only before the parts are
# read.  1 MiB leaves a margin; tests/test_envelope.py pins the behaviour.
_INLINE_MAX = 1 << 20


def envelope_parts(state, addr, port):
    """The global_model_update envelope as a list of buffers whose
    concatenation is its pickle (protocol 5): every contiguous fp32 tensor
    (on the GPU: one DMA each) is serialized from a pinned blob slot and
    handed to the pickler uncopied, so a socket can send the weights straight
    from the DMA target.  The caller holds ``LOCK`` until it is done with
    the parts (the next call reuses the slots).  Other tensors pickle as
    torch pickles them, from the host."""
    out = _Parts()
    model, settle = _fill(state)
    pickle.Pickler(out, protocol=5).dump({"type": "global_model_update", "model": model,
                                          "addr": addr, "port": port})
    settle()  # the large blobs' DMAs ran beside the pickler
    return out.parts


def dumps_state(state) -> bytes:
    """``pickle.dumps(state)`` for a trainer's local update (reference
    node/node.py:285) by the same route: each contiguous fp32 tensor DMA'd
    into a pinned blob slot of its own layout (the trainer's, apart from
    the global model's) and written once into the result.  ``pickle.loads``
    and the inbox's parser read it as they read torch's pickle."""
    with LOCK:
        out = _Parts()
        model, settle = _fill(state, purpose="update")
        pickle.Pickler(out, protocol=5).dump(model)
        settle()
        return b"".join(out.parts)


def _placeholders(state, purpose="global"):
    """The state_dict with each contiguous fp32 tensor replaced by a _Tensor
    over its freshly filled pinned blob slot (caller holds LOCK)."""
    model, settle = _fill(state, purpose)
    settle()
    return model


def _fill(state, purpose="global"):
    """_placeholders without waiting for the large slots: the DMAs of blobs
    the pickler copies (below _INLINE_MAX) are issued first and waited for
    here; the large ones after them, waited for by ``settle()`` -- so the
    pickler runs while they stream (caller holds LOCK)."""
    items = list(state.items())
    fast = [(k, t) for k, t in items if t.dtype == torch.float32 and t.is_contiguous()]
    model = collections.OrderedDict() if isinstance(state, collections.OrderedDict) else type(state)()
    slots = {}
    devices = []
    if fast:
        lay = _layout_for(purpose, fast)
        spans = list(zip(fast, lay.spans))
        devices = list({t.device for _, t in fast if t.is_cuda})
        inline_done = []
        if lay.dev is not None:  # one gather kernel, two DMAs
            with torch.cuda.device(lay.dev.device):
                _gather(lay, fast)
                if lay.inline_end:
                    lay.buf[:lay.inline_end].copy_(lay.dev[:lay.inline_end], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(lay.dev.device))
                inline_done.append(ev)
                if lay.inline_end < lay.buf.numel():
                    lay.buf[lay.inline_end:].copy_(lay.dev[lay.inline_end:], non_blocking=True)
        else:
            for large in (False, True):
                for (k, t), (a, p, e) in spans:
                    if (e - a >= _INLINE_MAX) == large and t.numel():
                        lay.buf[p:e].copy_(t.detach().reshape(-1).view(torch.uint8), non_blocking=t.is_cuda)
                if not large:
                    for d in devices:
                        ev = torch.cuda.Event()
                        ev.record(torch.cuda.current_stream(d))
                        inline_done.append(ev)
        for ev in inline_done:
            ev.synchronize()
        slots = {k: (t, lay.mv[a:e]) for (k, t), (a, _, e) in spans}

    def settle():
        for d in devices:
            torch.cuda.current_stream(d).synchronize()
    for k, t in items:
        if k in slots:
            src, mv = slots[k]
            model[k] = _Tensor(_Blob(mv), tuple(src.shape), tuple(src.stride()))
        else:
            model[k] = t.detach()  # pickled by torch, as the reference pickles it
    return model, settle


_LAND_TILE = 4096  # == P2P_LAND_TILE
_LAND_SEG = np.dtype([("src_off", "<u8"), ("dst", "<u8"), ("n", "<i8"), ("tile_begin", "<i8")])


def _gather(lay, fast):
    """Every fp32 tensor into its payload slot of the device image, one
    p2p_land_segments_f32 launch (K5's landing kernel as a gather: the
    sources are offsets from the lowest tensor address).  The segment table
    is built and uploaded when the tensors' addresses change (a model's
    parameters keep theirs across rounds)."""
    from .. import _native as N
    from .. import ops

    ptrs = tuple(t.data_ptr() for _, t in fast)
    if lay.gather is None or lay.gather[0] != ptrs:
        live = [(t.data_ptr(), t.numel(), p) for (_, t), (_, p, _) in zip(fast, lay.spans) if t.numel()]
        table = None
        base = span = ntiles = 0
        if live:
            base = min(a for a, _, _ in live)
            span = max(a + 4 * n for a, n, _ in live) - base
            tab = np.zeros(len(live), dtype=_LAND_SEG)
            tab["src_off"] = [a - base for a, _, _ in live]
            tab["dst"] = [lay.dev.data_ptr() + p for _, _, p in live]
            n_arr = np.array([n for _, n, _ in live], dtype=np.int64)
            tab["n"] = n_arr
            t_arr = -(-n_arr // _LAND_TILE)
            tab["tile_begin"][1:] = np.cumsum(t_arr)[:-1]
            ntiles = int(t_arr.sum())
            table = torch.from_numpy(tab.view(np.uint8).copy()).to(lay.dev.device)
        lay.gather = (ptrs, table, base, span, len(live), ntiles)
    _, table, base, span, nseg, ntiles = lay.gather
    if nseg:
        N.check(N.lib().p2p_land_segments_f32(base, span, table.data_ptr(), nseg, ntiles,
                                              N.stream_handle(lay.dev.device)), "p2p_land_segments_f32")


def global_model_envelope(state, addr, port) -> bytes:
    """The envelope as one bytes object: ``pickle.loads`` gives what the
    reference's ``pickle.dumps({"type": "global_model_update", "model":
    state, "addr": addr, "port": port})`` gives (one copy of the weights,
    into the result)."""
    with LOCK:
        return b"".join(envelope_parts(state, addr, port))
