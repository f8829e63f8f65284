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
    restricted stack machine over the opcodes torch emits (protocols 2-5)
    that resolves only the tensor-rebuild / legacy-storage callables and
    OrderedDict, parses the legacy storage blobs with the same machine
    (magic, header pickles, raw little-endian payload), checks every tensor
    view against its storage, and hands the payloads out as memoryview
    slices of the message -- no copy.  Anything else in the stream, and any
    malformed byte, raises ``pickle.UnpicklingError`` -- unlike the
    reference's ``pickle.loads`` on network bytes.  The stdlib unpickler is
    never run on peer bytes (its memo array lets a LONG_BINPUT index
    allocate gigabytes).
  * ``DeviceInbox.land`` copies the fp32 tensors of one update into row k of a
    preallocated [K_max, N] fp32 slab on the GPU -- through a pinned staging
    row, or, for a message received into the inbox's pinned buffers
    (``DeviceInbox.recv``), as the raw message bytes in one DMA and a landing
    kernel that places the payloads -- and returns a state_dict whose
    tensors are views of that row (the shape ``received_models`` expects,
    node/node.py:138).  The aggregation kernels then read K contiguous rows.

The values are bit-identical to ``pickle.loads`` (tests/test_inbox.py pins
this on torch-produced pickles of the reference's message shapes).
"""
from __future__ import annotations

import ctypes
import os
import pickle
import re
import struct
import threading
from collections import OrderedDict, deque
from dataclasses import dataclass

import numpy as np
import torch

from .._native import host_extension
from ..utils import digests

# torch legacy serialization (torch/serialization.py _legacy_save): magic
# number pickle, protocol-version pickle, sys_info pickle, the object pickle
# (storages as persistent ids), the storage-key list pickle, then per key an
# int64 element count and the raw bytes.
_LEGACY_MAGIC = 0x1950A86A20F9469CFC6C
# numpy has no bfloat16: a BFloat16Storage payload is held as its uint16 bit
# patterns (no other storage type maps to uint16) and materialised as a
# torch.bfloat16 view of them (RawTensor.tensor).
_STORAGE_DTYPES = {
    "FloatStorage": np.float32, "DoubleStorage": np.float64, "HalfStorage": np.float16,
    "BFloat16Storage": np.uint16, "LongStorage": np.int64, "IntStorage": np.int32, "ShortStorage": np.int16,
    "CharStorage": np.int8, "ByteStorage": np.uint8, "BoolStorage": np.bool_,
}
_TORCH_DTYPES = {np.float32: torch.float32, np.float64: torch.float64, np.float16: torch.float16,
                 np.uint16: torch.bfloat16, np.int64: torch.int64, np.int32: torch.int32, np.int16: torch.int16,
                 np.int8: torch.int8, np.uint8: torch.uint8, np.bool_: torch.bool}


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

    def tensor(self, device=None) -> torch.Tensor:
        """A torch tensor holding a copy of the payload, of the storage's
        dtype (bfloat16 from its bit patterns), on ``device`` (default: the
        storage's own location, as ``pickle.loads`` restores it)."""
        dev = device_of_location(self.storage.location) if device is None else device
        t = torch.from_numpy(np.array(self.array()))
        if self.storage.dtype is np.uint16:
            t = t.view(torch.bfloat16)
        return t if str(dev) == "cpu" else t.to(dev)


_LOCATION = re.compile(r"cpu|cuda(?::(\d{1,4}))?")


def device_of_location(location: str) -> str:
    """A peer's storage location as a device this process has: 'cpu', or
    'cuda' / 'cuda:<i>' with i below the visible device count (torch's own
    restore raises RuntimeError for a missing device).  Anything else raises
    pickle.UnpicklingError, the documented error for a peer's malformed
    bytes.  Checked where a tensor is materialised: the parsers
    (this module's and wire.cpp's, which must agree) keep the string, and a
    landed update's tensors go to the inbox's device whatever it names."""
    m = _LOCATION.fullmatch(location) if isinstance(location, str) else None
    if m is None:
        raise pickle.UnpicklingError(f"unsupported storage location {location!r}")
    if location != "cpu":
        i = int(m.group(1) or 0)
        if i >= torch.cuda.device_count():
            raise pickle.UnpicklingError(f"storage location {location!r}: no such device here")
    return location


class _Mark:
    pass


_MARK = _Mark()

# what malformed bytes make the stack machine raise (converted to
# pickle.UnpicklingError at the parser boundary)
_MALFORMED = (KeyError, IndexError, ValueError, TypeError, AttributeError, UnicodeDecodeError,
              struct.error, RecursionError, OverflowError, MemoryError)


def _run_pickle(mv: memoryview, pos: int, *, min_proto: int, resolve_global, persistent_load=None):
    """Restricted pickle stack machine over mv[pos:]: runs ONE pickle up to
    its STOP and returns (object, position after STOP).

    Only the opcodes torch emits for a state_dict and for the header pickles
    of a legacy storage blob (protocols 2-5) are accepted.  Globals resolve
    through ``resolve_global(module, name)`` (an allow-list); REDUCE calls
    only what that returned.  Byte strings come back as memoryview slices of
    mv (no copy).  The memo is a dict (a LONG_BINPUT with a huge index costs
    nothing, unlike the C unpickler's memo array) and every length field is
    checked against the end of the buffer."""
    n = len(mv)
    stack: list = []
    memo: dict = {}

    def need(p, k):  # bytes [p, p+k) must exist
        if k < 0 or p + k > n:
            raise pickle.UnpicklingError("truncated pickle")

    def le(p, k):
        need(p, k)
        return int.from_bytes(mv[p:p + k], "little")

    def blob(p, k):
        need(p, k)
        return mv[p:p + k]

    def pop_mark():  # in place: the rest of the stack is never copied
        for i in range(len(stack) - 1, -1, -1):
            if stack[i] is _MARK:
                items = stack[i + 1:]
                del stack[i:]
                return items
        raise pickle.UnpicklingError("MARK not found")

    while pos < n:
        op = mv[pos]
        pos += 1
        if op == 0x94:          # MEMOIZE
            memo[len(memo)] = stack[-1]
        elif op == 0x4B:          # BININT1
            stack.append(mv[pos])
            pos += 1
        elif op == 0x71:          # BINPUT
            memo[mv[pos]] = stack[-1]
            pos += 1
        elif op == 0x58:          # BINUNICODE
            k = le(pos, 4)
            stack.append(str(blob(pos + 4, k), "utf-8"))
            pos += 4 + k
        elif op == 0x8C:          # SHORT_BINUNICODE
            k = mv[pos]
            stack.append(str(blob(pos + 1, k), "utf-8"))
            pos += 1 + k
        elif op == 0x52:          # REDUCE
            args = stack.pop()
            fn = stack[-1]
            if not isinstance(fn, _Callable) or not isinstance(args, tuple):
                raise pickle.UnpicklingError("REDUCE of something that is not an allowed global")
            stack[-1] = fn(*args)
        elif op == 0x28:          # MARK
            stack.append(_MARK)
        elif op == 0x68:          # BINGET
            stack.append(memo[mv[pos]])
            pos += 1
        elif op == 0x85:          # TUPLE1
            stack[-1] = (stack[-1],)
        elif op == 0x74:          # TUPLE
            items = pop_mark()  # rebinds `stack`: take the items first
            stack.append(tuple(items))
        elif op == 0x42:          # BINBYTES
            k = le(pos, 4)
            stack.append(blob(pos + 4, k))
            pos += 4 + k
        elif op == 0x89:          # NEWFALSE
            stack.append(False)
        elif op == 0x29:          # EMPTY_TUPLE
            stack.append(())
        elif op == 0x2E:          # STOP
            return stack.pop(), pos
        elif op == 0x80:            # PROTO
            if mv[pos] < min_proto:
                raise pickle.UnpicklingError(f"pickle protocol {mv[pos]} (< {min_proto}) is not accepted")
            pos += 1
        elif op == 0x95:          # FRAME (8-byte length; frames are inline)
            need(pos, 8)
            pos += 8
        elif op == 0x7D:          # EMPTY_DICT
            stack.append({})
        elif op == 0x5D:          # EMPTY_LIST
            stack.append([])
        elif op == 0x72:          # LONG_BINPUT
            memo[le(pos, 4)] = stack[-1]
            pos += 4
        elif op == 0x6A:          # LONG_BINGET
            stack.append(memo[le(pos, 4)])
            pos += 4
        elif op == 0x43:          # SHORT_BINBYTES
            k = mv[pos]
            stack.append(blob(pos + 1, k))
            pos += 1 + k
        elif op == 0x8E:          # BINBYTES8
            k = le(pos, 8)
            stack.append(blob(pos + 8, k))
            pos += 8 + k
        elif op == 0x4D:          # BININT2
            stack.append(le(pos, 2))
            pos += 2
        elif op == 0x4A:          # BININT (signed)
            stack.append(int.from_bytes(blob(pos, 4), "little", signed=True))
            pos += 4
        elif op == 0x8A:          # LONG1
            k = mv[pos]
            stack.append(int.from_bytes(blob(pos + 1, k), "little", signed=True))
            pos += 1 + k
        elif op == 0x88:          # NEWTRUE
            stack.append(True)
        elif op == 0x4E:          # NONE
            stack.append(None)
        elif op == 0x86:          # TUPLE2
            b = stack.pop()
            stack[-1] = (stack[-1], b)
        elif op == 0x87:          # TUPLE3
            c = stack.pop()
            b = stack.pop()
            stack[-1] = (stack[-1], b, c)
        elif op == 0x93:          # STACK_GLOBAL
            name = stack.pop()
            module = stack.pop()
            if not (isinstance(module, str) and isinstance(name, str)):
                raise pickle.UnpicklingError("STACK_GLOBAL needs two strings")
            stack.append(resolve_global(module, name))
        elif op == 0x63:          # GLOBAL (text: module\nname\n)
            e1 = bytes(mv[pos:pos + 256]).index(b"\n")
            module = str(mv[pos:pos + e1], "ascii")
            e2 = bytes(mv[pos + e1 + 1:pos + e1 + 257]).index(b"\n")
            name = str(mv[pos + e1 + 1:pos + e1 + 1 + e2], "ascii")
            pos += e1 + e2 + 2
            stack.append(resolve_global(module, name))
        elif op == 0x51:          # BINPERSID
            if persistent_load is None:
                raise pickle.UnpicklingError("persistent ids are not accepted here")
            stack[-1] = persistent_load(stack[-1])
        elif op == 0x62:          # BUILD (OrderedDict metadata: set attributes)
            state = stack.pop()
            inst = stack[-1]
            if isinstance(state, dict) and isinstance(inst, OrderedDict):
                # torch sets only `_metadata`; any other attribute could
                # shadow the dict's methods (items / values) on the instance
                if set(state) - {"_metadata"}:
                    raise pickle.UnpicklingError("unexpected attributes on a state_dict")
                inst.__dict__.update(state)
            elif state is not None:
                raise pickle.UnpicklingError("unexpected BUILD")
        elif op == 0x73:          # SETITEM
            v = stack.pop()
            k = stack.pop()
            dict.__setitem__(stack[-1], k, v)
        elif op == 0x75:          # SETITEMS
            items = pop_mark()
            d = stack[-1]
            for i in range(0, len(items), 2):
                dict.__setitem__(d, items[i], items[i + 1])
        elif op == 0x61:          # APPEND
            v = stack.pop()
            list.append(stack[-1], v)
        elif op == 0x65:          # APPENDS
            items = pop_mark()
            list.extend(stack[-1], items)
        else:
            raise pickle.UnpicklingError(f"opcode 0x{op:02x} is not accepted in a peer update")
    raise pickle.UnpicklingError("truncated pickle")


class _Callable:
    """An allow-listed global (the only thing REDUCE may call)."""

    def __init__(self, fn, name):
        self.fn, self.name = fn, name

    def __call__(self, *args):
        return self.fn(*args)


class _StorageType(str):
    """A torch.<X>Storage global of a storage record, kept as its name."""


def _storage_global(module, name):
    if module == "torch" and name in _STORAGE_DTYPES:
        return _StorageType(name)
    raise pickle.UnpicklingError(f"unexpected global {module}.{name} in a tensor storage blob")


def _no_global(module, name):
    raise pickle.UnpicklingError(f"unexpected global {module}.{name} in a tensor storage header")


# The magic / protocol-version / sys_info pickles that open every legacy blob
# of one sender are the same bytes: the last prefix that parsed and passed the
# checks is matched byte for byte instead of re-parsed (3 of the 5 pickles).
_HEADER_OK = b""


def parse_legacy_storage(blob) -> RawStorage:
    """One torch legacy storage blob (torch/serialization.py _legacy_save): the
    magic-number, protocol-version and sys_info pickles (no globals allowed),
    the storage record (a persistent id naming the storage type, key,
    location and element count), the key-list pickle, then an int64 count
    and the raw little-endian payload.  Every pickle runs on the restricted
    machine: the blob is the peer's."""
    if not isinstance(blob, (memoryview, bytes, bytearray)):
        raise pickle.UnpicklingError("storage blob must be bytes")
    mv = memoryview(blob).cast("B")
    global _HEADER_OK
    ok = _HEADER_OK
    if ok and mv[:len(ok)] == ok:
        # the same three header pickles as a blob already validated below:
        # identical bytes, identical (accepted) values
        pos = len(ok)
    else:
        magic, pos = _run_pickle(mv, 0, min_proto=2, resolve_global=_no_global)
        if type(magic) is not int or magic != _LEGACY_MAGIC:
            raise pickle.UnpicklingError("not a torch legacy storage blob (magic)")
        f_ver, pos = _run_pickle(mv, pos, min_proto=2, resolve_global=_no_global)
        if type(f_ver) is not int or f_ver != 1001:
            raise pickle.UnpicklingError(f"unsupported legacy protocol version {f_ver!r}")
        sys_info, pos = _run_pickle(mv, pos, min_proto=2, resolve_global=_no_global)
        if not isinstance(sys_info, dict) or sys_info.get("little_endian") is not True:
            raise pickle.UnpicklingError("storage blob is not little-endian")
        if pos <= 256:
            _HEADER_OK = bytes(mv[:pos])
    pids = []

    def persistent_load(pid):
        pids.append(pid)
        return None

    _, pos = _run_pickle(mv, pos, min_proto=2, resolve_global=_storage_global, persistent_load=persistent_load)
    if len(pids) != 1 or not isinstance(pids[0], tuple) or len(pids[0]) < 5 or pids[0][0] != "storage":
        raise pickle.UnpicklingError("storage blob without exactly one storage record")
    pid = pids[0]
    _, stype, key, location, numel = pid[:5]
    if not isinstance(stype, _StorageType) or type(numel) is not int or numel < 0 or not isinstance(key, str):
        raise pickle.UnpicklingError("malformed storage record")
    if len(pid) > 5 and pid[5] is not None:
        raise pickle.UnpicklingError("storage views are not supported")
    keys, pos = _run_pickle(mv, pos, min_proto=2, resolve_global=_no_global)
    if keys != [key]:
        raise pickle.UnpicklingError("expected exactly one storage per blob")
    dt = _STORAGE_DTYPES[stype]
    if pos + 8 > len(mv):
        raise pickle.UnpicklingError("truncated storage blob")
    (count,) = struct.unpack_from("<q", mv, pos)
    nbytes = count * np.dtype(dt).itemsize
    if count != numel or pos + 8 + nbytes != len(mv):
        raise pickle.UnpicklingError("storage payload size mismatch")
    return RawStorage(dt, int(numel), mv[pos + 8:pos + 8 + nbytes], str(location))


def _is_index(x) -> bool:
    return type(x) is int and x >= 0


def _rebuild_tensor_v2(storage, offset, size, stride, requires_grad=False, hooks=None, metadata=None):
    """The view a peer claims must lie inside its storage (torch's own
    set_() refuses it otherwise): non-negative integer offset, sizes and
    strides, and the last addressed element below storage.numel.  Without
    this an as_strided view would read past the message buffer."""
    if not isinstance(storage, RawStorage):
        raise pickle.UnpicklingError("tensor without a storage")
    if not (isinstance(size, tuple) and isinstance(stride, tuple) and len(size) == len(stride)):
        raise pickle.UnpicklingError("tensor size / stride must be tuples of the same length")
    if not (_is_index(offset) and all(map(_is_index, size)) and all(map(_is_index, stride))):
        raise pickle.UnpicklingError("tensor offset, sizes and strides must be non-negative integers")
    if all(size):  # non-empty: the furthest element must exist
        last = offset + sum((s - 1) * st for s, st in zip(size, stride))
        if last >= storage.numel:
            raise pickle.UnpicklingError(f"tensor view ends at element {last}, storage holds {storage.numel}")
        # A state_dict tensor is dense: a view repeating elements (a zero
        # stride, or more elements than its storage holds) would make a
        # few-byte message expand into an arbitrarily large copy.
        if any(st == 0 and s > 1 for s, st in zip(size, stride)):
            raise pickle.UnpicklingError("tensor view with a zero stride")
        numel = 1
        for s in size:
            numel *= s
        if numel > storage.numel - offset:
            raise pickle.UnpicklingError(f"tensor view of {numel} elements over {storage.numel - offset}")
    elif offset > storage.numel:
        raise pickle.UnpicklingError("tensor offset past the end of its storage")
    return RawTensor(storage, offset, size, stride)


def _ordered_dict(*args):
    if args:
        raise pickle.UnpicklingError("OrderedDict with arguments")
    return OrderedDict()


# The globals a pickled state_dict of tensors needs (torch's tensor pickling:
# _rebuild_tensor_v2 over a legacy-format storage blob; the OrderedDict of
# state_dict()).  Nothing else resolves.
_UPDATE_GLOBALS = {
    ("torch._utils", "_rebuild_tensor_v2"): _Callable(_rebuild_tensor_v2, "_rebuild_tensor_v2"),
    ("torch.storage", "_load_from_bytes"): _Callable(parse_legacy_storage, "_load_from_bytes"),
    ("collections", "OrderedDict"): _Callable(_ordered_dict, "OrderedDict"),
}


def _update_global(module, name):
    fn = _UPDATE_GLOBALS.get((module, name))
    if fn is None:
        raise pickle.UnpicklingError(f"refusing to load global {module}.{name} from a peer update")
    return fn


def _is_tensor_dict(obj) -> bool:
    """A dict whose values are all tensors (dict.values, not obj.values: the
    method lookup must not go through attributes a pickle could set)."""
    return isinstance(obj, dict) and all(isinstance(v, RawTensor) for v in dict.values(obj))


# the same machine in C++ (csrc/wire.cpp), built beside the HIP library; the
# product parses with it (NativeUnavailable at import when it is not built).
# The Python machine above stays as its differential reference in the tests
# (ZeroCopyParser(native=False)).
_wire = host_extension("_wire")


class ZeroCopyParser:
    """Reader for the pickled state_dict of a peer update (reference
    node/node.py:285; pickle protocols 3-5).  Runs the restricted stack
    machine: byte strings are memoryview slices of the message buffer -- the
    tensor payloads are never copied -- only the three globals above resolve,
    and anything else, or any malformed byte, raises
    ``pickle.UnpicklingError`` (so a listener that catches only that cannot
    be killed by a peer's bytes).

    ``native`` (default) runs the machine in C++
    (``csrc/wire.cpp``, without the GIL) -- the same opcodes, globals and
    checks as the Python machine below, which the tests hold it to; it
    returns the same RawTensor / RawStorage views."""

    def __init__(self, data, native: bool | None = None):
        self.mv = memoryview(data).cast("B")
        self.native = True if native is None else native

    def parse(self) -> dict:
        if self.native:
            entries, storages = _wire.parse_update(self.mv)
            mv = self.mv
            st = [RawStorage(_STORAGE_DTYPES[t], numel, mv[off:off + nb], loc) for t, numel, off, nb, loc in storages]
            return OrderedDict((key, RawTensor(st[si], o, size, stride)) for key, si, o, size, stride in entries)
        try:
            obj, _ = _run_pickle(self.mv, 0, min_proto=3, resolve_global=_update_global)
        except pickle.UnpicklingError:
            raise
        except _MALFORMED as e:
            raise pickle.UnpicklingError(f"malformed peer update: {type(e).__name__}: {e}") from e
        if not _is_tensor_dict(obj):
            raise pickle.UnpicklingError("a peer update must be a dict of tensors")
        return OrderedDict(dict.items(obj))  # a fresh dict: no attributes the pickle set


def recv_exact_into(conn, buf: memoryview) -> int:
    """Fill buf from the socket; returns the bytes received (< len on EOF)."""
    got = 0
    while got < len(buf):
        n = conn.recv_into(buf[got:], len(buf) - got)
        if n == 0:
            break
        got += n
    return got


_RECV_STEP = 64 << 20  # pageable receive grows in steps of this size (bytes arrive first)


def recv_message(conn) -> bytearray | None:
    """One length-prefixed message (reference node/node.py:99-112 framing:
    4-byte big-endian length, then the pickle), received linearly.  Returns
    None if the peer closed early (the reference then drops the message)."""
    hdr = bytearray(4)
    if recv_exact_into(conn, memoryview(hdr)) != 4:
        return None
    return recv_body(conn, int.from_bytes(hdr, "big"))


def recv_body(conn, n: int) -> bytearray | None:
    """The n message bytes after the length prefix, in pageable memory that
    grows as bytes arrive (from 64 MiB, doubling), like the reference's
    buffer: a bogus length claims no memory up front.  None on early close."""
    data = bytearray(min(n, _RECV_STEP))
    got = 0
    while True:
        got += recv_exact_into(conn, memoryview(data)[got:])
        if got < len(data):
            return None
        if got == n:
            return data
        data += bytes(min(len(data), n - len(data)))


_REF_LOCK = threading.Lock()


def _pinned_bytes(n: int) -> torch.Tensor:
    return torch.empty(n, dtype=torch.uint8, pin_memory=True)


class _PinnedBuffer:
    """A page-locked host buffer of the inbox's pool.  ``refs`` counts the
    live ``PinnedMessage`` handles on it (the received message and the
    windows cut from it); at zero it goes back to the pool, and it is handed
    out again only after the last DMA and digest that read it are done."""

    def __init__(self, capacity: int, pool):
        self.buf = _pinned_bytes(max(int(capacity), 1))
        self.pool = pool      # the DeviceInbox whose pool it returns to
        self.refs = 0
        self.event = None     # the host-to-device copy that last read buf
        self.digest = None    # the SHA-256 future that reads buf

    @property
    def capacity(self) -> int:
        return self.buf.numel()

    def wait_idle(self) -> None:
        if self.event is not None:
            self.event.synchronize()
            self.event = None
        if self.digest is not None:
            self.digest.result()
            self.digest = None


class PinnedMessage:
    """A handle on a received message in page-locked host memory
    (``DeviceInbox.recv`` / ``message_buffer``), or on a window of one
    (``window``, e.g. the serialized update inside the reference's envelope,
    node/node.py:133).  ``DeviceInbox.land`` moves it to the device in ONE
    DMA, as bytes, and the landing kernel (csrc/land.hip) places its fp32
    payloads in the slab row: the host never copies a payload byte.

    The bytes stay valid, and the buffer stays out of the pool, while ANY
    handle on it is alive: ``release()`` (or garbage collection of the
    handle) gives the handle up, and when the last one goes the buffer
    returns to the inbox's pool.  ``land`` does not release: a listener can
    still read ``view()`` (the echo's bytes, utils/broadcast.py:14,23) after
    landing.  Pickled, a handle is its bytes (the echo envelope carries them,
    utils/broadcast.py:18-24)."""

    def __init__(self, root: _PinnedBuffer, start: int, nbytes: int):
        self.root, self.start, self.nbytes = root, int(start), int(nbytes)
        self.buf = root.buf
        with _REF_LOCK:
            root.refs += 1
        self._held = True

    def view(self) -> memoryview:
        if not self._held:
            raise ValueError("the message was released (its buffer may hold another message)")
        return memoryview(self.buf.numpy())[self.start:self.start + self.nbytes]

    def __len__(self) -> int:
        return self.nbytes

    def __bytes__(self) -> bytes:
        return bytes(self.view())

    def __reduce__(self):
        return (bytes, (bytes(self.view()),))

    def window(self, part: memoryview) -> "PinnedMessage":
        """``part`` (a slice of ``view()``) as a message of its own that shares
        this buffer (and holds it): ``land`` reads it in place."""
        base = self.buf.data_ptr()
        at = np.frombuffer(part, dtype=np.uint8).ctypes.data - base if len(part) else self.start
        if not (self.start <= at and at + len(part) <= self.start + self.nbytes):
            raise ValueError("window outside the message")
        return PinnedMessage(self.root, at, len(part))

    def release(self, _collected: bool = False) -> None:
        """Give this handle up (idempotent)."""
        with _REF_LOCK:
            if not self._held:
                return
            self._held = False
            self.root.refs -= 1
            last = self.root.refs == 0
        if last and self.root.pool is not None:
            if _collected:
                # from __del__: the garbage collector can run this on a thread
                # that holds the inbox's lock, so no lock here -- the buffer
                # is queued and the pool takes it at its next hand-out
                self.root.pool._return_later(self.root)
            else:
                self.root.pool._release(self.root)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.release()
        return False

    def __del__(self):
        try:
            self.release(_collected=True)
        except Exception:  # interpreter shutdown
            pass


def _detached(v):
    """A restricted-machine value with every byte string (a memoryview of
    the receive buffer) copied out as bytes and every tensor view
    materialised as a torch tensor on its storage's location (what
    ``pickle.loads`` gives), at any depth."""
    if isinstance(v, memoryview):
        return bytes(v)
    if isinstance(v, RawTensor):
        return v.tensor()
    if isinstance(v, list):
        return [_detached(x) for x in v]
    if isinstance(v, tuple):
        return tuple(_detached(x) for x in v)
    if isinstance(v, dict):
        d = OrderedDict() if isinstance(v, OrderedDict) else {}
        for a, b in dict.items(v):
            d[_detached(a)] = _detached(b)
        meta = getattr(v, "__dict__", {}).get("_metadata") if isinstance(v, OrderedDict) else None
        if meta is not None:  # BUILD's only attribute: load_state_dict reads it (node.py:244)
            d._metadata = _detached(meta)
        return d
    return v


def _envelope_global(module, name):
    """Globals an envelope may name: only those of a pickled state_dict of
    tensors (the 'global_model_update' model, aggregation.py:70), each
    resolved to the restricted machine's own callable (the legacy storage
    blob is parsed by parse_legacy_storage, never by torch.load)."""
    fn = _UPDATE_GLOBALS.get((module, name))
    if fn is None:
        raise pickle.UnpicklingError(f"refusing to load global {module}.{name} from a peer message")
    return fn


def decode_envelope(mv: memoryview):
    """A peer's message envelope (node/node.py:112) on the restricted
    machine: (object, plain) where plain is the decoded dict with byte
    strings still memoryviews of ``mv`` and tensors still RawTensor views.
    Every message the reference sends -- 'connect', 'model_update', 'echo',
    'ready', 'sup' (str / int / bytes / None / lists and dicts of them) and
    'global_model_update' (a state_dict of tensors) -- decodes here; anything
    else, or any malformed byte, raises ``pickle.UnpicklingError``.  No
    stdlib unpickler ever runs on peer bytes."""
    try:
        obj, pos = _run_pickle(mv, 0, min_proto=2, resolve_global=_envelope_global)
    except pickle.UnpicklingError:
        raise
    except _MALFORMED as e:
        raise pickle.UnpicklingError(f"malformed peer message: {type(e).__name__}: {e}") from e
    if not isinstance(obj, dict) or pos != len(mv):
        raise pickle.UnpicklingError("a peer message must be one pickled dict")
    return obj


def _dense(rt: "RawTensor") -> bool:
    """C-contiguous view (dims of size 1 may carry any stride)."""
    want = 1
    for n, st in zip(reversed(rt.size), reversed(rt.stride)):
        if n != 1 and st != want:
            return False
        want *= n
    return True


def _address(mv: memoryview) -> int:
    """Host address of a (non-empty) buffer slice: through ctypes for the
    writable pinned buffers (~0.3 us), numpy otherwise."""
    try:
        return ctypes.addressof(ctypes.c_char.from_buffer(mv))
    except TypeError:
        return np.frombuffer(mv, dtype=np.uint8).ctypes.data


_LAND_TILE = 4096  # == P2P_LAND_TILE
_LAND_SEG = np.dtype([("src_off", "<u8"), ("dst", "<u8"), ("n", "<i8"), ("tile_begin", "<i8")])


class LandedUpdate(OrderedDict):
    """What DeviceInbox.land returns: {key: tensor} in the update's key order,
    the fp32 entries views of ONE slab row.  It is frozen (every mutator
    raises TypeError), so the aggregator can trust that the entries listed in
    ``slab_keys`` are still slab[row, offset : offset + numel] and build its
    kernel table from (slab, row, layout) without inspecting each tensor
    (ops.aggregate_slab_rows_)."""

    def __init__(self, items, inbox: "DeviceInbox", row: int, slab_keys: frozenset):
        super().__init__(items)
        self.inbox, self.row, self.slab_keys = inbox, row, slab_keys
        self._frozen = True

    def _refuse(self, *a, **k):
        if getattr(self, "_frozen", False):
            raise TypeError("a landed update is read-only (its tensors are slab views)")

    def __setitem__(self, key, value):
        self._refuse()
        super().__setitem__(key, value)

    def __delitem__(self, key):
        self._refuse()
        super().__delitem__(key)

    def clear(self):
        self._refuse()

    def pop(self, *a):
        self._refuse()

    def popitem(self, *a, **k):
        self._refuse()

    def setdefault(self, *a):
        self._refuse()

    def update(self, *a, **k):
        self._refuse()

    def move_to_end(self, *a, **k):
        self._refuse()

    def __ior__(self, other):
        self._refuse()

    def __reduce__(self):
        # a plain OrderedDict of copies: pickling a slab view would carry the
        # whole slab (torch pickles a view's entire storage)
        return (OrderedDict, ([(k, v.clone()) for k, v in self.items()],))


ROW_ALIGN = 64  # fp32 elements (256 B) per tensor offset in a slab row
# The chunk layout (round 5): every key on a 1024-float boundary and the row
# pitch whole 8192-float tiles, so FedAvg can read the rows as flat peers on
# the split kernel (ops._rows_entry, include/p2pdl.h p2p_fedavg_split_rows_f32)
# -- taken when it pads the row by at most CHUNK_PAD_MAX.
ROW_CHUNK, ROW_TILE, CHUNK_PAD_MAX = 1024, 8192, 0.05


class _Consuming:
    """DeviceInbox.consuming(): the landing lock held around a launch."""

    __slots__ = ("inbox", "stream")

    def __init__(self, inbox, stream):
        self.inbox, self.stream = inbox, stream

    def __enter__(self):
        from .. import _native as N

        ib, stream = self.inbox, self.stream
        ib._lock.acquire()
        try:
            events = [e for e in ib._events if e is not None]
            raw = stream.cuda_stream if stream is not None else N.stream_handle(ib.device)
            if events or raw not in ib._consumers:
                stream = stream or torch.cuda.current_stream(ib.device)
                for ev in events:
                    stream.wait_event(ev)
                ib._consumers.setdefault(raw, (stream, torch.cuda.Event()))
        except BaseException:
            ib._lock.release()
            raise
        return self

    def __exit__(self, *exc):
        self.inbox._lock.release()
        return False


class DeviceInbox:
    """[K_max, N] fp32 slab on the GPU for the updates of one round.

    ``template`` is the receiving node's state_dict (reference: its
    self.model); its fp32 entries fix the row layout (key order, offsets).
    ``land(serialized, k)`` parses one serialized update and lands it in row
    k; ``reset()`` starts a new round.  Non-fp32 entries (e.g. int64
    counters) are materialised as ordinary small device tensors."""

    def __init__(self, template: dict, k_max: int, device=None, max_message_bytes: int | None = None,
                 pool_bytes: int | None = None):
        self.device = torch.device(device) if device is not None else next(
            (t.device for t in template.values() if t.is_cuda), torch.device("cuda", torch.cuda.current_device()))
        # 256-B aligned offsets (and row pitch): every tensor view starts a
        # 128-B HBM line, as a separate allocation would -- a 16-B aligned
        # view straddles one more line per kernel tile.  The chunk layout
        # (1024-float offsets, whole-tile pitch) when it costs <= 5% of the row.
        f32 = [(key, t) for key, t in template.items() if t.dtype == torch.float32]

        def place(align, pitch_to):
            lay, off = OrderedDict(), 0
            for key, t in f32:
                lay[key] = (off, tuple(t.shape), t.numel())
                off += -(-t.numel() // align) * align
            return lay, -(-off // pitch_to) * pitch_to if off else 0

        self.layout, self.row = place(ROW_ALIGN, ROW_ALIGN)
        chunked, crow = place(ROW_CHUNK, ROW_TILE)
        if crow <= (1 + CHUNK_PAD_MAX) * self.row:
            self.layout, self.row = chunked, crow
        self.k_max = int(k_max)
        self.slab = torch.empty((self.k_max, self.row), dtype=torch.float32, device=self.device)
        self._stage = [torch.empty(self.row, dtype=torch.float32, pin_memory=True) for _ in range(2)]
        self._events = [None, None]
        self._dmsg = [None, None]  # device copies of pinned messages (landing kernel input)
        self._views = [{} for _ in range(self.k_max)]  # row k: {key: slab view}
        # A message of up to max_message_bytes is received into pinned memory
        # (default: the template's payload plus the pickle framing -- about 325
        # B per tensor, SURVEY.md §3D -- and 1 MiB of envelope / extra keys);
        # a longer one into pageable memory.  The pool of free pinned buffers
        # holds at most pool_bytes (default: two per row of the slab).
        extra = sum(t.numel() * t.element_size() for t in template.values() if t.dtype != torch.float32)
        self.max_message_bytes = int(max_message_bytes if max_message_bytes is not None else
                                     4 * self.row + extra + 1024 * len(template) + (1 << 20))
        self.pool_bytes = int(pool_bytes if pool_bytes is not None else 2 * self.k_max * self.max_message_bytes)
        self._pinned_free = []     # _PinnedBuffer pool
        self._returned = deque()   # buffers of finalised handles, pooled at the next hand-out
        self._consumers = {}       # stream handle -> (stream, event): streams whose kernels read the slab
        self._digests = {}
        self.count = 0
        # land() is called from the listener threads (one per connection,
        # reference node/node.py:89): row reservation and the staging ->
        # device sequence are serialised; parsing runs outside the lock.
        self._lock = threading.Lock()

    def reset(self) -> None:
        with self._lock:
            self.count = 0
            self._digests = {}

    def land(self, serialized, k: int | None = None, digest: bool = False) -> dict:
        """Parse one serialized update and copy it to slab row k (next free row
        by default).  Returns {key: tensor} in the update's key order, fp32
        entries as views of the slab row -- bit-identical to pickle.loads.
        ``serialized`` as bytes-like: the payloads go message buffer ->
        pinned staging row (one memcpy, split across a thread pool) -> device
        (one DMA).  As a ``PinnedMessage`` (``recv`` / ``message_buffer``):
        the whole message -> device in one DMA, then one landing kernel
        places the payloads (csrc/land.hip) -- no host copy of the payloads.

        digest=True also starts SHA-256 of the serialized bytes -- what the
        tester signs in its echo (node/node.py:144 -> utils/crypto.py:54-57)
        -- on a hashing thread, overlapped with the parse, the staging copy
        and the DMA of this update and the next; ``digest(k)`` returns it,
        and so does the process's digest cache (utils/digests.py) for this
        same object: the echo's ``sign_data(key, serialized)`` (reference
        utils/broadcast.py:14, unchanged) reuses it.  The buffer must not
        change until then.  (Host SHA-NI: one message is one serial chain,
        ~2.4 GB/s on a host core vs ~33 MB/s on one GPU lane -- DESIGN.md §3
        K3.)  Landing does not release a ``PinnedMessage``: its bytes stay
        valid until every handle on its buffer is released."""
        pinned = serialized if isinstance(serialized, PinnedMessage) else None
        if pinned is not None:
            serialized = pinned.view()
        # SHA-256 of the bytes on a hashing thread, registered in the process's
        # digest cache under this very object: sign_data / verify_signature of
        # it (utils/crypto.py) then pick it up instead of hashing again
        fut = digests.digest_async(pinned if pinned is not None else serialized) if digest else None
        if pinned is not None and fut is not None:
            pinned.root.digest = fut  # the pool hands the buffer out again only after it
        raw = ZeroCopyParser(serialized).parse()
        with self._lock:
            if k is None:
                k = self.count
            if not 0 <= k < self.k_max:
                raise IndexError(f"slab row {k} out of range (k_max={self.k_max})")
            self.count = max(self.count, k + 1)
            if fut is not None:
                self._digests[k] = fut
            else:  # a digest of the row's previous bytes must not outlive them
                self._digests.pop(k, None)
            if pinned is None:
                return self._land_locked(raw, k)
            got = self._land_pinned_locked(pinned, raw, k)
            return got if got is not None else self._land_locked(raw, k)

    def message_buffer(self, nbytes: int) -> PinnedMessage:
        """A pinned buffer for a message of ``nbytes`` (the smallest free one
        of the pool that fits, or a new one), as a handle; the buffer returns
        to the pool when the handle and every window of it are released."""
        nbytes = int(nbytes)
        with self._lock:
            self._drain_returned_locked()
            fits = [p for p in self._pinned_free if p.capacity >= nbytes]
            root = min(fits, key=lambda p: p.capacity) if fits else None
            if root is not None:
                self._pinned_free.remove(root)
        if root is None:
            root = _PinnedBuffer(nbytes, self)
        root.wait_idle()
        return PinnedMessage(root, 0, nbytes)

    def _release(self, root: _PinnedBuffer) -> None:
        """A buffer with no live handle: back to the pool while the pool holds
        at most pool_bytes, freed otherwise."""
        with self._lock:
            self._pool_locked(root)

    def _pool_locked(self, root: _PinnedBuffer) -> None:
        if any(p is root for p in self._pinned_free):
            return
        if sum(p.capacity for p in self._pinned_free) + root.capacity <= self.pool_bytes:
            self._pinned_free.append(root)

    def _return_later(self, root: _PinnedBuffer) -> None:
        """_release without the lock (deque.append is atomic): for handles
        the garbage collector finalises."""
        self._returned.append(root)

    def _drain_returned_locked(self) -> None:
        while self._returned:
            self._pool_locked(self._returned.popleft())

    def recv(self, conn):
        """``recv_message`` into a pinned buffer of this inbox: the 4-byte
        big-endian length (node/node.py:99-112 framing), then the message, as
        a ``PinnedMessage``.  A message longer than ``max_message_bytes``
        arrives in pageable memory instead (a ``bytearray`` that grows as
        bytes arrive), so a peer's length field cannot pin host memory.
        None if the peer closed early (the buffer goes back to the pool)."""
        hdr = bytearray(4)
        if recv_exact_into(conn, memoryview(hdr)) != 4:
            return None
        n = int.from_bytes(hdr, "big")
        if n > self.max_message_bytes:
            return recv_body(conn, n)
        m = self.message_buffer(n)
        if recv_exact_into(conn, m.view()) != m.nbytes:
            m.release()
            return None
        return m

    def consuming(self, stream=None) -> "_Consuming":
        """The block in which a caller enqueues a kernel that reads slab rows
        on ``stream`` (default: the current stream of the slab's device),
        under the landing lock: the stream waits for every row copy ``land``
        has issued (``order_after_landing``) and is registered as a consumer
        (``slab_consumed``) BEFORE the kernel is queued, and no ``land`` on
        another thread runs in between -- one that ran before is covered by
        the wait, one that runs after records its own wait on this stream
        after the kernel (registering only after the launch let
        a land in that window overwrite rows the kernel was reading).  A
        plain class, not a generator context: cfg1's whole call is ~12 us."""
        return _Consuming(self, stream)

    def slab_consumed(self, stream=None) -> None:
        """Record that a kernel just issued on ``stream`` (default: the current
        stream of the slab's device) reads slab rows: every later ``land``
        makes its own stream wait for that kernel before it overwrites a row
        (aggregation.py calls this after each launch over landed updates).
        The wait is set up by ``land``, not here: a land on another stream
        records an event on each consuming stream at that moment -- after
        every kernel issued on it so far -- and waits for it; a land on the
        consuming stream itself is ordered by the stream.  So the per-call
        cost of an aggregation is one dict lookup (a hipEventRecord per call
        measured ~4.7 us of cfg1's ~14 us call, tools/prof_cfg1_parts.py)."""
        from .. import _native as N

        raw = stream.cuda_stream if stream is not None else N.stream_handle(self.device)
        if raw in self._consumers:
            return
        with self._lock:
            if raw not in self._consumers:
                self._consumers[raw] = (stream or torch.cuda.current_stream(self.device), torch.cuda.Event())

    def _wait_rows_free(self, stream) -> None:
        """Make ``stream`` wait for every kernel issued so far on the
        streams that read the slab (under self._lock)."""
        for raw, (consumer, ev) in self._consumers.items():
            if raw != stream.cuda_stream:
                ev.record(consumer)
                stream.wait_event(ev)

    def order_after_landing(self, stream=None) -> None:
        """Make ``stream`` (default: the current stream of the slab's device)
        wait for the row copies issued by ``land`` -- they run on the landing
        thread's stream -- so a kernel launched on it reads the landed bytes.
        Device-side waits only; the host does not block."""
        with self._lock:
            events = [e for e in self._events if e is not None]
        if not events:
            return
        stream = stream or torch.cuda.current_stream(self.device)
        for ev in events:
            stream.wait_event(ev)

    def digest(self, k: int) -> bytes:
        """SHA-256 of the bytes landed in row k with ``land(..., digest=True)``
        (waits for the hashing thread)."""
        with self._lock:
            fut = self._digests.get(k)
        if fut is None:
            raise KeyError(f"slab row {k} was not landed with digest=True")
        return fut.result()

    def _land_locked(self, raw, k: int) -> dict:
        s = k & 1
        if self._events[s] is not None:
            self._events[s].synchronize()  # the staging row is free again
        stage = self._stage[s].numpy()
        row = self.slab[k]
        out = OrderedDict()
        jobs = []
        for key, rt in dict.items(raw):
            lay = self.layout.get(key)
            if lay is not None and rt.storage.dtype is np.float32:
                off, shape, n = lay
                if rt.size != shape:
                    raise RuntimeError(f"update key {key}: shape {rt.size} != {shape}")
                jobs.append((stage[off:off + n], rt))
            else:  # not part of the fp32 slab: a small tensor of its own
                out[key] = rt.tensor(self.device)
        _copy_all(jobs)
        with torch.cuda.device(self.device):
            self._wait_rows_free(torch.cuda.current_stream())
            row.copy_(self._stage[s], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._events[s] = ev
        slab_keys = []
        for key in raw:
            if key in out:
                continue
            out[key] = self._row_view(k, key)
            slab_keys.append(key)
        return LandedUpdate(((key, out[key]) for key in raw), self, k, frozenset(slab_keys))

    def open_envelope(self, msg) -> dict:
        """The reference's message envelope decoded (replaces pickle.loads at
        node/node.py:112) from what ``recv`` returned.

        A plain envelope of a ``model_update`` (a pickled dict: 'type', 'addr',
        'port' and the serialized update under 'model', :130-135) is parsed by
        the restricted machine (no globals) and 'model' comes back as a
        ``PinnedMessage`` window of the receive buffer, so ``land`` reads the
        update where it arrived; every other bytes value is real ``bytes``.
        Every other message -- 'global_model_update' carries a state_dict of
        tensors (aggregation.py:70), 'echo' / 'ready' / 'sup' carry
        signatures and whole updates as bytes -- decodes to the values the
        reference's ``pickle.loads`` gives (plain objects; tensors on their
        storage's location), on the same restricted machine
        (``decode_envelope``): no stdlib unpickler runs on a peer's bytes, and
        a message it does not accept raises ``pickle.UnpicklingError``.  The
        handle ``msg`` is consumed: its buffer returns to the pool once no
        window of it is alive (at once when none escapes)."""
        try:
            if not isinstance(msg, PinnedMessage):  # pageable (over the pinned cap)
                return _detached(decode_envelope(memoryview(msg).cast("B")))
            try:
                obj = decode_envelope(msg.view())
                if not (dict.get(obj, "type") == "model_update" and isinstance(dict.get(obj, "model"), memoryview)):
                    return _detached(obj)
                return {k: (msg.window(v) if k == "model" else _detached(v)) for k, v in dict.items(obj)}
            finally:
                msg.release()
        except RecursionError as e:  # a nesting too deep, or a cycle (memo), to copy out
            raise pickle.UnpicklingError("peer message nests too deeply") from e

    def _land_pinned_locked(self, msg: PinnedMessage, raw, k: int):
        """K5 device path: the message bytes in one DMA, then one landing
        kernel over a segment table (payload byte offset -> row offset).
        None (nothing issued) when an fp32 view is not dense: the staging
        path handles strided views."""
        from .. import _native as N
        from .. import ops

        base = msg.buf.data_ptr() + msg.start
        row = self.slab[k]
        row_ptr = row.data_ptr()
        out = OrderedDict()
        segs = []
        for key, rt in dict.items(raw):
            lay = self.layout.get(key)
            if lay is not None and rt.storage.dtype is np.float32:
                off, shape, n = lay
                if rt.size != shape:
                    raise RuntimeError(f"update key {key}: shape {rt.size} != {shape}")
                if not _dense(rt):
                    return None
                if n:
                    src = _address(rt.storage.data) - base + 4 * rt.offset
                    # the parser already bounds every view by its storage and
                    # every storage by the message; a layout that still points
                    # outside the message fails here, loudly, instead of landing
                    # the kernel's zero fill
                    if src < 0 or src + 4 * n > msg.nbytes:
                        raise pickle.UnpicklingError(f"update key {key}: payload [{src}, {src + 4 * n}) "
                                                     f"outside the {msg.nbytes}-byte message")
                    segs.append((src, row_ptr + 4 * off, n))
            else:  # not part of the fp32 slab: a small tensor of its own
                out[key] = rt.tensor(self.device)
        s = k & 1
        with torch.cuda.device(self.device):
            stream = torch.cuda.current_stream()
            if self._events[s] is not None:
                stream.wait_event(self._events[s])  # the last kernel that read _dmsg[s]
            self._wait_rows_free(stream)  # the last aggregation that read the rows
            d = self._dmsg[s]
            if d is None or d.numel() < msg.nbytes:
                d = self._dmsg[s] = torch.empty(max(msg.nbytes, 1 << 20), dtype=torch.uint8, device=self.device)
            d[:msg.nbytes].copy_(msg.buf[msg.start:msg.start + msg.nbytes], non_blocking=True)
            msg.root.event = torch.cuda.Event()
            msg.root.event.record()
            if segs:
                tab = np.zeros(len(segs), dtype=_LAND_SEG)
                tab["src_off"] = [a for a, _, _ in segs]
                tab["dst"] = [b for _, b, _ in segs]
                n_arr = np.array([n for _, _, n in segs], dtype=np.int64)
                tab["n"] = n_arr
                t_arr = -(-n_arr // _LAND_TILE)
                tab["tile_begin"][1:] = np.cumsum(t_arr)[:-1]
                dtab = ops._RING.to_device(tab.view(np.uint8), self.device)
                N.check(N.lib().p2p_land_segments_f32(d.data_ptr(), msg.nbytes, dtab.data_ptr(), len(segs),
                                                      int(t_arr.sum()), stream.cuda_stream),
                        "p2p_land_segments_f32")
            ev = torch.cuda.Event()
            ev.record()
            self._events[s] = ev
        slab_keys = []
        for key in raw:
            if key in out:
                continue
            out[key] = self._row_view(k, key)
            slab_keys.append(key)
        return LandedUpdate(((key, out[key]) for key in raw), self, k, frozenset(slab_keys))

    def _row_view(self, k: int, key):
        """slab[k, off : off + n].view(shape) for a template key, built once
        per (row, key): the slab is never reallocated, so the view is the
        same every round (62 tensor slices per ResNet-18 update otherwise)."""
        views = self._views[k]
        v = views.get(key)
        if v is None:
            off, shape, n = self.layout[key]
            v = views[key] = self.slab[k, off:off + n].view(shape)
        return v

    def view(self, k: int) -> LandedUpdate:
        """Row k as a landed update holding every fp32 key of the template
        (for rows filled on the device, e.g. by synthetic generators)."""
        if not 0 <= k < self.k_max:
            raise IndexError(f"slab row {k} out of range (k_max={self.k_max})")
        row = self.slab[k]
        items = [(key, row[off:off + n].view(shape)) for key, (off, shape, n) in self.layout.items()]
        return LandedUpdate(items, self, k, frozenset(self.layout))


_POOL = None
_POOL_LOCK = threading.Lock()


def _copy_all(jobs) -> None:
    """dst[:] = src for (dst, RawTensor) pairs; large copies on a thread pool
    (numpy releases the GIL while copying)."""
    global _POOL
    big = [j for j in jobs if j[0].size >= (1 << 18)]
    small = [j for j in jobs if j[0].size < (1 << 18)]
    if big:
        with _POOL_LOCK:  # land() runs on several listener threads
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
