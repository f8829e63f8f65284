"""Receive peer updates straight into a device slab.

Reference ``Node.handle_connection`` (node/node.py:97-141) receives a message
with ``data += packet`` in 4 KiB pieces (:104-109, quadratic in the message
size: a 100 MB update is copied ~25k times), ``pickle.loads`` the envelope
(:112) and then the serialized update (:135), and appends the resulting
state_dict to ``received_models`` (:138).  Unpickling a tensor re-runs
``torch.load`` on a legacy-format blob per tensor and, for a CUDA sender,
allocates and copies every tensor to the GPU separately.

Here:
  * ``recv_message`` reads the 4-byte length and ``recv_into`` one
    preallocated buffer (linear);
  * ``ZeroCopyParser`` decodes the serialized update WITHOUT executing it: a
    restricted stack machine over the opcodes torch emits (protocols 3-5)
    that resolves only the tensor-rebuild / legacy-storage callables and
    OrderedDict, parses the legacy storage blobs itself (magic, header
    pickles, raw little-endian payload) and hands the payloads out as
    memoryview slices of the message -- no copy.  Anything else in the stream
    raises ``pickle.UnpicklingError`` -- unlike the reference's
    ``pickle.loads`` on network bytes.  (``UpdateParser`` is the same
    restriction on top of the C unpickler, which copies each payload once.)
  * ``DeviceInbox.land`` copies the fp32 tensors of one update into row k of a
    preallocated [K_max, N] fp32 slab on the GPU through a pinned staging row
    -- one host-to-device copy per update -- and returns a state_dict whose
    tensors are views of that row (the shape ``received_models`` expects,
    node/node.py:138).  The aggregation kernels then read K contiguous rows.

The values are bit-identical to ``pickle.loads`` (tests/test_inbox.py pins
this on torch-produced pickles of the reference's message shapes).
"""
from __future__ import annotations

import os
import pickle
import struct
from collections import OrderedDict
from dataclasses import dataclass

import numpy as np
import torch

# torch legacy serialization (torch/serialization.py _legacy_save): magic
# number pickle, protocol-version pickle, sys_info pickle, the object pickle
# (storages as persistent ids), the storage-key list pickle, then per key an
# int64 element count and the raw bytes.
_LEGACY_MAGIC = 0x1950A86A20F9469CFC6C
_STORAGE_DTYPES = {
    "FloatStorage": np.float32, "DoubleStorage": np.float64, "HalfStorage": np.float16,
    "BFloat16Storage": None, "LongStorage": np.int64, "IntStorage": np.int32, "ShortStorage": np.int16,
    "CharStorage": np.int8, "ByteStorage": np.uint8, "BoolStorage": np.bool_,
}
_TORCH_DTYPES = {np.float32: torch.float32, np.float64: torch.float64, np.float16: torch.float16,
                 np.int64: torch.int64, np.int32: torch.int32, np.int16: torch.int16, np.int8: torch.int8,
                 np.uint8: torch.uint8, np.bool_: torch.bool}


@dataclass
class RawStorage:
    dtype: type          # numpy scalar type
    numel: int
    data: memoryview     # raw little-endian payload inside the message buffer
    location: str        # 'cpu', 'cuda:0', ...


@dataclass
class RawTensor:
    storage: RawStorage
    offset: int
    size: tuple
    stride: tuple

    @property
    def numel(self) -> int:
        return int(np.prod(self.size)) if self.size else 1

    def array(self) -> np.ndarray:
        """numpy view of the payload (no copy for contiguous tensors)."""
        base = np.frombuffer(self.storage.data, dtype=self.storage.dtype, count=self.storage.numel)
        if not self.size:
            return base[self.offset:self.offset + 1].reshape(())
        item = base.itemsize
        return np.lib.stride_tricks.as_strided(base[self.offset:], shape=self.size,
                                               strides=tuple(s * item for s in self.stride), writeable=False)


class _Reader:
    """Minimal read-only file over a buffer: pickle pulls only what it parses
    (io.BytesIO would first copy the whole message)."""

    def __init__(self, buf):
        self.mv = memoryview(buf).cast("B")
        self.pos = 0

    def read(self, n=-1):
        end = len(self.mv) if n is None or n < 0 else min(len(self.mv), self.pos + n)
        out = self.mv[self.pos:end].tobytes()
        self.pos = end
        return out

    def readinto(self, b):
        n = min(len(b), len(self.mv) - self.pos)
        b[:n] = self.mv[self.pos:self.pos + n]
        self.pos += n
        return n

    def readline(self):
        end = self.pos
        while end < len(self.mv):
            chunk = self.mv[end:end + 256].tobytes()
            i = chunk.find(b"\n")
            if i >= 0:
                end += i + 1
                break
            end += len(chunk)
        return self.read(end - self.pos)

    def tell(self):
        return self.pos


class _StorageHeader(pickle.Unpickler):
    """Unpickles the header pickles of one legacy storage blob."""

    def find_class(self, module, name):
        if module == "torch" and name in _STORAGE_DTYPES:
            return name  # the storage type, as its name
        raise pickle.UnpicklingError(f"unexpected global {module}.{name} in a tensor storage blob")

    def persistent_load(self, pid):
        if not (isinstance(pid, tuple) and len(pid) >= 5 and pid[0] == "storage"):
            raise pickle.UnpicklingError(f"unexpected persistent id {pid!r}")
        self.pid = pid
        return pid


def parse_legacy_storage(blob) -> RawStorage:
    mv = memoryview(blob).cast("B")
    f = _Reader(mv)
    if pickle.Unpickler(f).load() != _LEGACY_MAGIC:
        raise pickle.UnpicklingError("not a torch legacy storage blob (magic)")
    f_ver = pickle.Unpickler(f).load()
    if f_ver != 1001:
        raise pickle.UnpicklingError(f"unsupported legacy protocol version {f_ver}")
    pickle.Unpickler(f).load()  # sys_info
    hdr = _StorageHeader(f)
    hdr.load()
    _, stype, key, location, numel = hdr.pid[:5]
    if len(hdr.pid) > 5 and hdr.pid[5] is not None:
        raise pickle.UnpicklingError("storage views are not supported")
    keys = _StorageHeader(f).load()
    if keys != [key]:
        raise pickle.UnpicklingError("expected exactly one storage per blob")
    dt = _STORAGE_DTYPES[stype]
    if dt is None:
        raise pickle.UnpicklingError(f"{stype} is not supported")
    pos = f.tell()
    (count,) = struct.unpack_from("<q", mv, pos)
    nbytes = count * np.dtype(dt).itemsize
    if count != numel or pos + 8 + nbytes != len(mv):
        raise pickle.UnpicklingError("storage payload size mismatch")
    return RawStorage(dt, int(numel), mv[pos + 8:pos + 8 + nbytes], str(location))


def _rebuild_tensor_v2(storage, offset, size, stride, requires_grad=False, hooks=None, metadata=None):
    if not isinstance(storage, RawStorage):
        raise pickle.UnpicklingError("tensor without a storage")
    return RawTensor(storage, int(offset), tuple(size), tuple(stride))


class UpdateParser(pickle.Unpickler):
    """Restricted unpickler for a pickled state_dict (reference node/node.py:285)."""

    _ALLOWED = {
        ("torch._utils", "_rebuild_tensor_v2"): _rebuild_tensor_v2,
        ("torch.storage", "_load_from_bytes"): parse_legacy_storage,
        ("collections", "OrderedDict"): OrderedDict,
    }

    def find_class(self, module, name):
        fn = self._ALLOWED.get((module, name))
        if fn is None:
            raise pickle.UnpicklingError(f"refusing to load global {module}.{name} from a peer update")
        return fn

    @classmethod
    def parse(cls, data) -> dict:
        obj = cls(_Reader(data)).load()
        if not isinstance(obj, dict) or not all(isinstance(v, RawTensor) for v in obj.values()):
            raise pickle.UnpicklingError("a peer update must be a dict of tensors")
        return obj


class _Mark:
    pass


_MARK = _Mark()


class ZeroCopyParser:
    """Restricted stack-machine reader for the pickled state_dict of a peer
    update (pickle protocols 3-5, the opcodes torch emits for a dict of
    tensors).  Byte strings are returned as memoryview slices of the message
    buffer -- the tensor payloads are never copied by the parser -- and only
    the globals of ``UpdateParser`` resolve; anything else raises
    ``pickle.UnpicklingError``."""

    def __init__(self, data):
        self.mv = memoryview(data).cast("B")

    def parse(self) -> dict:
        mv = self.mv
        n = len(mv)
        pos = 0
        stack: list = []
        memo: dict = {}
        u8 = lambda p: mv[p]  # noqa: E731
        le = lambda p, k: int.from_bytes(mv[p:p + k], "little")  # noqa: E731

        def pop_mark():
            nonlocal stack
            for i in range(len(stack) - 1, -1, -1):
                if stack[i] is _MARK:
                    items = stack[i + 1:]
                    stack = stack[:i]
                    return items
            raise pickle.UnpicklingError("MARK not found")

        while pos < n:
            op = mv[pos]
            pos += 1
            if op == 0x80:            # PROTO
                if mv[pos] < 3:
                    raise pickle.UnpicklingError(f"pickle protocol {mv[pos]} (< 3) is not accepted")
                pos += 1
            elif op == 0x95:          # FRAME (8-byte length; frames are inline)
                pos += 8
            elif op == 0x2E:          # STOP
                result = stack.pop()
                if not isinstance(result, dict) or not all(isinstance(v, RawTensor) for v in result.values()):
                    raise pickle.UnpicklingError("a peer update must be a dict of tensors")
                return result
            elif op == 0x28:          # MARK
                stack.append(_MARK)
            elif op == 0x7D:          # EMPTY_DICT
                stack.append({})
            elif op == 0x29:          # EMPTY_TUPLE
                stack.append(())
            elif op == 0x5D:          # EMPTY_LIST
                stack.append([])
            elif op == 0x94:          # MEMOIZE
                memo[len(memo)] = stack[-1]
            elif op == 0x71:          # BINPUT
                memo[mv[pos]] = stack[-1]
                pos += 1
            elif op == 0x72:          # LONG_BINPUT
                memo[le(pos, 4)] = stack[-1]
                pos += 4
            elif op == 0x68:          # BINGET
                stack.append(memo[mv[pos]])
                pos += 1
            elif op == 0x6A:          # LONG_BINGET
                stack.append(memo[le(pos, 4)])
                pos += 4
            elif op == 0x8C:          # SHORT_BINUNICODE
                k = mv[pos]
                stack.append(str(mv[pos + 1:pos + 1 + k], "utf-8"))
                pos += 1 + k
            elif op == 0x58:          # BINUNICODE
                k = le(pos, 4)
                stack.append(str(mv[pos + 4:pos + 4 + k], "utf-8"))
                pos += 4 + k
            elif op == 0x43:          # SHORT_BINBYTES
                k = mv[pos]
                stack.append(mv[pos + 1:pos + 1 + k])
                pos += 1 + k
            elif op == 0x42:          # BINBYTES
                k = le(pos, 4)
                stack.append(mv[pos + 4:pos + 4 + k])
                pos += 4 + k
            elif op == 0x8E:          # BINBYTES8
                k = le(pos, 8)
                stack.append(mv[pos + 8:pos + 8 + k])
                pos += 8 + k
            elif op == 0x4B:          # BININT1
                stack.append(mv[pos])
                pos += 1
            elif op == 0x4D:          # BININT2
                stack.append(le(pos, 2))
                pos += 2
            elif op == 0x4A:          # BININT (signed)
                stack.append(int.from_bytes(mv[pos:pos + 4], "little", signed=True))
                pos += 4
            elif op == 0x8A:          # LONG1
                k = mv[pos]
                stack.append(int.from_bytes(mv[pos + 1:pos + 1 + k], "little", signed=True))
                pos += 1 + k
            elif op == 0x89:          # NEWFALSE
                stack.append(False)
            elif op == 0x88:          # NEWTRUE
                stack.append(True)
            elif op == 0x4E:          # NONE
                stack.append(None)
            elif op == 0x85:          # TUPLE1
                stack[-1] = (stack[-1],)
            elif op == 0x86:          # TUPLE2
                b = stack.pop()
                stack[-1] = (stack[-1], b)
            elif op == 0x87:          # TUPLE3
                c = stack.pop()
                b = stack.pop()
                stack[-1] = (stack[-1], b, c)
            elif op == 0x74:          # TUPLE
                items = pop_mark()  # rebinds `stack`: take the items first
                stack.append(tuple(items))
            elif op == 0x93:          # STACK_GLOBAL
                name = stack.pop()
                module = stack.pop()
                stack.append(self._global(module, name))
            elif op == 0x63:          # GLOBAL (text: module\nname\n)
                e1 = bytes(mv[pos:pos + 256]).index(b"\n")
                module = str(mv[pos:pos + e1], "ascii")
                e2 = bytes(mv[pos + e1 + 1:pos + e1 + 257]).index(b"\n")
                name = str(mv[pos + e1 + 1:pos + e1 + 1 + e2], "ascii")
                pos += e1 + e2 + 2
                stack.append(self._global(module, name))
            elif op == 0x52:          # REDUCE
                args = stack.pop()
                fn = stack[-1]
                stack[-1] = fn(*args)
            elif op == 0x62:          # BUILD (OrderedDict metadata: set attributes)
                state = stack.pop()
                inst = stack[-1]
                if isinstance(state, dict) and isinstance(inst, OrderedDict):
                    inst.__dict__.update({k: v for k, v in state.items() if isinstance(k, str)})
                elif state is not None:
                    raise pickle.UnpicklingError("unexpected BUILD")
            elif op == 0x73:          # SETITEM
                v = stack.pop()
                k = stack.pop()
                stack[-1][k] = v
            elif op == 0x75:          # SETITEMS
                items = pop_mark()
                d = stack[-1]
                for i in range(0, len(items), 2):
                    d[items[i]] = items[i + 1]
            elif op == 0x61:          # APPEND
                v = stack.pop()
                stack[-1].append(v)
            elif op == 0x65:          # APPENDS
                items = pop_mark()
                stack[-1].extend(items)
            else:
                raise pickle.UnpicklingError(f"opcode 0x{op:02x} is not accepted in a peer update")
        raise pickle.UnpicklingError("truncated pickle")

    @staticmethod
    def _global(module, name):
        fn = UpdateParser._ALLOWED.get((module, name))
        if fn is None:
            raise pickle.UnpicklingError(f"refusing to load global {module}.{name} from a peer update")
        return fn


def recv_exact_into(conn, buf: memoryview) -> int:
    """Fill buf from the socket; returns the bytes received (< len on EOF)."""
    got = 0
    while got < len(buf):
        n = conn.recv_into(buf[got:], len(buf) - got)
        if n == 0:
            break
        got += n
    return got


def recv_message(conn) -> bytearray | None:
    """One length-prefixed message (reference node/node.py:99-112 framing:
    4-byte big-endian length, then the pickle), received linearly.  Returns
    None if the peer closed early (the reference then drops the message)."""
    hdr = bytearray(4)
    if recv_exact_into(conn, memoryview(hdr)) != 4:
        return None
    n = int.from_bytes(hdr, "big")
    data = bytearray(n)
    if recv_exact_into(conn, memoryview(data)) != n:
        return None
    return data


class DeviceInbox:
    """[K_max, N] fp32 slab on the GPU for the updates of one round.

    ``template`` is the receiving node's state_dict (reference: its
    self.model); its fp32 entries fix the row layout (key order, offsets).
    ``land(serialized, k)`` parses one serialized update and lands it in row
    k; ``reset()`` starts a new round.  Non-fp32 entries (e.g. int64
    counters) are materialised as ordinary small device tensors."""

    def __init__(self, template: dict, k_max: int, device=None):
        self.device = torch.device(device) if device is not None else next(
            (t.device for t in template.values() if t.is_cuda), torch.device("cuda", torch.cuda.current_device()))
        self.layout = OrderedDict()
        off = 0
        for key, t in template.items():
            if t.dtype == torch.float32:
                # 16-B aligned offsets so every row and every tensor view is DMA-friendly
                self.layout[key] = (off, tuple(t.shape), t.numel())
                off += -(-t.numel() // 4) * 4
        self.row = off
        self.k_max = int(k_max)
        self.slab = torch.empty((self.k_max, self.row), dtype=torch.float32, device=self.device)
        self._stage = [torch.empty(self.row, dtype=torch.float32, pin_memory=True) for _ in range(2)]
        self._events = [None, None]
        self.count = 0

    def reset(self) -> None:
        self.count = 0

    def land(self, serialized, k: int | None = None) -> dict:
        """Parse one serialized update and copy it to slab row k (next free row
        by default).  Returns {key: tensor} in the update's key order, fp32
        entries as views of the slab row -- bit-identical to pickle.loads.
        The payloads go message buffer -> pinned staging row (one memcpy,
        split across a thread pool) -> device (one DMA)."""
        raw = ZeroCopyParser(serialized).parse()
        if k is None:
            k = self.count
        if not 0 <= k < self.k_max:
            raise IndexError(f"slab row {k} out of range (k_max={self.k_max})")
        self.count = max(self.count, k + 1)
        s = k & 1
        if self._events[s] is not None:
            self._events[s].synchronize()  # the staging row is free again
        stage = self._stage[s].numpy()
        row = self.slab[k]
        out = OrderedDict()
        jobs = []
        for key, rt in raw.items():
            lay = self.layout.get(key)
            if lay is not None and rt.storage.dtype is np.float32:
                off, shape, n = lay
                if rt.size != shape:
                    raise RuntimeError(f"update key {key}: shape {rt.size} != {shape}")
                jobs.append((stage[off:off + n], rt))
            else:  # not part of the fp32 slab: a small tensor of its own
                out[key] = torch.from_numpy(np.array(rt.array())).to(self.device)
        _copy_all(jobs)
        with torch.cuda.device(self.device):
            row.copy_(self._stage[s], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._events[s] = ev
        for key in raw:
            if key in out:
                continue
            off, shape, n = self.layout[key]
            out[key] = row[off:off + n].view(shape)
        return OrderedDict((key, out[key]) for key in raw)


_POOL = None


def _copy_all(jobs) -> None:
    """dst[:] = src for (dst, RawTensor) pairs; large copies on a thread pool
    (numpy releases the GIL while copying)."""
    global _POOL
    big = [j for j in jobs if j[0].size >= (1 << 18)]
    small = [j for j in jobs if j[0].size < (1 << 18)]
    if big:
        if _POOL is None:
            from concurrent.futures import ThreadPoolExecutor
            _POOL = ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1))
        pieces = []
        for dst, rt in big:  # split the large tensors into ~1M-element pieces
            src = rt.array().reshape(-1)
            for a in range(0, dst.size, 1 << 20):
                pieces.append((dst[a:a + (1 << 20)], src[a:a + (1 << 20)]))
        list(_POOL.map(lambda p: np.copyto(p[0], p[1]), pieces))
    for dst, rt in small:
        dst[:] = rt.array().reshape(-1)
