"""SHA-256 of serialized updates, computed once per distinct message.

The reference hashes the same serialized update inside every
``ECDSA(SHA256())`` call (utils/crypto.py:54-57 sign, :92-96 verify): 72
SHA-256 passes over 3 distinct messages per round in the default
configuration (node/node.py:145,155,187-206).  This module
keeps the digests this process has already computed, so ``sign_data`` /
``verify_signature`` keep the reference's call signatures and still hash a
message only the first time its bytes are seen:

  * a hit by IDENTITY -- the same ``bytes`` object, or the same
    ``PinnedMessage`` window (node/inbox.py) that ``DeviceInbox.land(...,
    digest=True)`` hashed at arrival -- costs a dict lookup;
  * a hit by CONTENT -- another object with equal bytes, e.g. the ready
    message's copy of an update this node received earlier (node/node.py:175)
    -- costs one memcmp (~10 GB/s on a host core, 4x cheaper than SHA-NI);
  * a miss is hashed on the host (``hashlib``: one message is one serial
    chain, ~2.4 GB/s with SHA-NI, against ~33 MB/s for one GPU lane chain --
    DESIGN.md §3 K3), or, for a batch of many distinct messages, by the GPU
    batch kernel (``digest_many``; the boundary is measured).

Only immutable references are kept: ``bytes`` objects (held, bounded by
count and bytes, least recently used evicted first) and ``PinnedMessage``
windows (weakly: a window's buffer cannot return to the pool while it is
alive, and the entry dies with it).  Equal digests are SHA-256 of equal
bytes by construction, so a cache hit can never change a verification
result.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import threading
import weakref
from collections import OrderedDict, deque
from concurrent.futures import Future

import numpy as np

_libc = ctypes.CDLL(None)
_libc.memcmp.restype = ctypes.c_int
_libc.memcmp.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]

_PROBE = 32  # bytes of head and tail in the content key


def _buffer(data) -> memoryview:
    """Byte view of bytes / bytearray / memoryview / PinnedMessage."""
    if _is_window(data):
        return data.view()
    return memoryview(data).cast("B")


def _address(mv: memoryview) -> int:
    return np.frombuffer(mv, dtype=np.uint8).ctypes.data


def _same_bytes(a: memoryview, b: memoryview) -> bool:
    n = len(a)
    if n != len(b):
        return False
    return n == 0 or _libc.memcmp(_address(a), _address(b), n) == 0


def _is_window(data) -> bool:
    return type(data).__name__ == "PinnedMessage" and hasattr(data, "root")


class DigestCache:
    """Digests by identity and by content (see the module docstring)."""

    def __init__(self, max_entries: int = 256, max_bytes: int = 1 << 30):
        self.max_entries, self.max_bytes = int(max_entries), int(max_bytes)
        self._by_id: "OrderedDict[int, tuple]" = OrderedDict()  # id -> (ref, key)
        self._by_key: dict = {}  # content key -> {id: (ref, digest or Future)}
        self._held = 0  # bytes of strongly held `bytes` objects
        self._dead = deque()  # weak references whose windows died
        self._lock = threading.Lock()
        self.hits_identity = self.hits_content = self.misses = 0

    @staticmethod
    def _key(mv: memoryview):
        n = len(mv)
        return n, bytes(mv[:_PROBE]), bytes(mv[max(0, n - _PROBE):])

    @staticmethod
    def _alive(ref):
        return ref() if isinstance(ref, weakref.ref) else ref

    def clear(self) -> None:
        with self._lock:
            self._dead.clear()
            self._by_id.clear()
            self._by_key.clear()
            self._held = 0

    def __len__(self) -> int:
        with self._lock:
            self._purge_locked()
            return len(self._by_id)

    def _purge_locked(self) -> None:
        while self._dead:
            ref = self._dead.popleft()
            for oid, (r, _) in list(self._by_id.items()):
                if r is ref:
                    self._drop_locked(oid)
                    break

    def _drop_locked(self, oid: int) -> None:
        ref, key = self._by_id.pop(oid)
        bucket = self._by_key.get(key)
        if bucket is not None:
            bucket.pop(oid, None)
            if not bucket:
                del self._by_key[key]
        if isinstance(ref, bytes):
            self._held -= len(ref)

    def put(self, data, digest) -> None:
        """Remember ``digest`` (32 bytes, or a Future of them) for ``data``
        when ``data`` is immutable for as long as the entry lives."""
        if isinstance(data, bytes):
            ref = data
        elif _is_window(data):
            if not data._held:
                return
            # the entry is purged lazily: the callback may run (garbage
            # collection) on a thread inside this cache's lock
            ref = weakref.ref(data, self._dead.append)
        else:
            return  # mutable: looked up, never kept
        key = self._key(_buffer(data))
        oid = id(data)
        with self._lock:
            self._purge_locked()
            if oid in self._by_id:
                self._drop_locked(oid)
            self._by_id[oid] = (ref, key)
            self._by_key.setdefault(key, {})[oid] = (ref, digest)
            if isinstance(ref, bytes):
                self._held += len(ref)
            while self._by_id and (len(self._by_id) > self.max_entries or self._held > self.max_bytes):
                self._drop_locked(next(iter(self._by_id)))

    def get(self, data):
        """The digest (or its Future) of ``data``'s bytes if known, else None."""
        oid = id(data)
        mv = _buffer(data)
        key = self._key(mv)
        with self._lock:
            self._purge_locked()
            bucket = self._by_key.get(key)
            if not bucket:
                return None
            ent = bucket.get(oid)
            if ent is not None and self._alive(ent[0]) is data and not (_is_window(data) and not data._held):
                self._by_id.move_to_end(oid)
                self.hits_identity += 1
                return ent[1]
            cands = [(self._alive(r), d) for r, d in bucket.values()]
        for obj, d in cands:
            if obj is None or (_is_window(obj) and not obj._held):
                continue  # a released window: its buffer may hold another message by now
            if _same_bytes(mv, _buffer(obj)):
                with self._lock:
                    self.hits_content += 1
                self.put(data, d)  # the next lookup of this object is by identity
                return d
        return None


CACHE = DigestCache()
_POOL = None
_POOL_PREFIX = "p2p-sha256"
_POOL_LOCK = threading.Lock()


def hash_threads() -> int:
    """Hashing threads: this process's CPU affinity, capped by
    OMP_NUM_THREADS when the environment sets it (the GPU box exports 16, one
    GPU's share of its host cores; os.cpu_count() there counts the whole
    machine).  bench.py's hashlib baseline uses the same rule
    (oracle/cpu_baseline.py host_threads), so the two rates compare like for
    like."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    env = os.environ.get("OMP_NUM_THREADS", "")
    return min(aff, int(env)) if env.isdigit() and int(env) > 0 else aff


def hash_pool():
    """Host hashing threads (hashlib releases the GIL on large buffers)."""
    global _POOL
    with _POOL_LOCK:
        if _POOL is None:
            from concurrent.futures import ThreadPoolExecutor

            _POOL = ThreadPoolExecutor(max_workers=hash_threads(), thread_name_prefix=_POOL_PREFIX)
        return _POOL


def _result(d) -> bytes:
    return d.result() if isinstance(d, Future) else d


def sha256_host(data) -> bytes:
    return hashlib.sha256(_buffer(data)).digest()


def digest_of(data) -> bytes:
    """SHA-256 of one message: from the cache, else hashed on the host once."""
    d = CACHE.get(data)
    if d is not None:
        return _result(d)
    with CACHE._lock:
        CACHE.misses += 1
    d = sha256_host(data)
    CACHE.put(data, d)
    return d


def digest_async(data) -> Future:
    """digest_of on a hashing thread (DeviceInbox.land(..., digest=True)):
    the Future is registered at once, so a sign / verify of the same object
    issued before the hash finishes waits for it instead of hashing again."""
    d = CACHE.get(data)
    if d is not None:
        if isinstance(d, Future):
            return d
        f = Future()
        f.set_result(d)
        return f
    with CACHE._lock:
        CACHE.misses += 1
    fut = hash_pool().submit(sha256_host, data)
    CACHE.put(data, fut)
    return fut


# The GPU batch kernel hashes every message on its own lane chain (~33 MB/s
# each, all in parallel); the host hashes one message per thread at ~2.4
# GB/s (SHA-NI).  For host-resident messages the GPU wins only for a batch of
# many short ones (measured boundary, DESIGN.md §3 K3,
# profiles/r04/digest_boundary.json): at least GPU_BATCH_MIN distinct
# messages, none longer than GPU_MAX_MESSAGE bytes.
GPU_BATCH_MIN = 256
GPU_MAX_MESSAGE = 16384
HOST_THREAD_MIN = 1 << 16  # shorter messages hash inline on the calling thread


def _gpu_batch_wins(msgs) -> bool:
    return len(msgs) >= GPU_BATCH_MIN and max(len(m) for m in msgs) <= GPU_MAX_MESSAGE


# Device-resident messages (cfg5: 256 x 100 MB in HBM): the same boundary.
# Off the GPU kernel's side they cross PCIe in STAGE-byte pieces into pinned
# buffers of the hashing thread that owns the message (two per thread, the
# next piece in flight on the thread's own stream while it hashes the last):
# the D2H (~50 GB/s) hides under the hashing (~2.4 GB/s per thread).
STAGE = 8 << 20
_TLS = threading.local()


def _staging(dev):
    st = getattr(_TLS, "stage", None)
    if st is None or st[0] != dev:
        import torch

        st = (dev, torch.cuda.Stream(dev), [torch.empty(STAGE, dtype=torch.uint8, pin_memory=True) for _ in range(2)],
              [torch.cuda.Event() for _ in range(2)])
        _TLS.stage = st
    return st


def _hash_device_message(msgs, off: int, n: int, ready) -> bytes:
    import torch

    _, stream, bufs, evs = _staging(msgs.device)
    stream.wait_event(ready)  # the messages as the caller's stream left them
    h = hashlib.sha256()
    pieces = [(o, min(STAGE, off + n - o)) for o in range(off, off + n, STAGE)]

    def issue(i):
        o, ln = pieces[i]
        with torch.cuda.stream(stream):
            bufs[i % 2][:ln].copy_(msgs[o:o + ln], non_blocking=True)
            evs[i % 2].record(stream)

    if pieces:
        issue(0)
    for i, (_, ln) in enumerate(pieces):
        if i + 1 < len(pieces):
            issue(i + 1)  # buffer (i + 1) % 2 held piece i - 1, hashed already
        evs[i % 2].synchronize()
        h.update(memoryview(bufs[i % 2].numpy())[:ln])
    return h.digest()


def digest_device_messages(msgs, offsets, lengths):
    """SHA-256 of K messages in one device uint8 buffer, as a (K, 32) uint8
    device tensor: the GPU batch kernel (``ops.sha256_batch_device``) for
    GPU_BATCH_MIN or more messages of at most GPU_MAX_MESSAGE bytes, else the
    host hashing threads with each message streamed over PCIe in STAGE-byte
    pieces (for long messages one host thread hashes ~70x
    faster than one GPU lane chain).  Synchronises on the host route."""
    import torch

    from .. import ops

    offsets, lengths = [int(o) for o in offsets], [int(x) for x in lengths]
    ops.check_message_spans(msgs, offsets, lengths)
    if len(offsets) >= GPU_BATCH_MIN and max(lengths, default=0) <= GPU_MAX_MESSAGE:
        return ops.sha256_batch_device(msgs, offsets, lengths)
    dev = msgs.device
    ready = torch.cuda.Event()
    ready.record(torch.cuda.current_stream(dev))
    if threading.current_thread().name.startswith(_POOL_PREFIX):  # a pool task waiting on the pool could deadlock
        ds = [_hash_device_message(msgs, o, n, ready) for o, n in zip(offsets, lengths)]
    else:
        ds = [f.result() for f in [hash_pool().submit(_hash_device_message, msgs, o, n, ready)
                                   for o, n in zip(offsets, lengths)]]
    out = np.frombuffer(b"".join(ds), dtype=np.uint8).reshape(len(offsets), 32)
    return torch.from_numpy(out.copy()).to(dev)


def digest_many(messages) -> list:
    """SHA-256 of every message, each distinct message hashed at most once:
    cached ones from the cache, the rest on the host threads or -- for
    GPU_BATCH_MIN or more of them -- in ONE launch of the GPU batch kernel
    (``ops.sha256_batch``)."""
    messages = list(messages)
    out = [None] * len(messages)
    todo = []  # (index, message) of cache misses
    for i, m in enumerate(messages):
        d = CACHE.get(m)
        if d is None:
            todo.append(i)
        else:
            out[i] = d
    if todo:
        uniq, slot, seen = [], {}, {}  # distinct misses: by identity, then by content
        for i in todo:
            m = messages[i]
            j = seen.get(id(m))
            if j is None:
                mv = _buffer(m)
                for j0 in seen.get(DigestCache._key(mv), ()):
                    if _same_bytes(mv, _buffer(uniq[j0])):
                        j = j0
                        break
                if j is None:
                    j = len(uniq)
                    uniq.append(m if isinstance(m, bytes) else bytes(mv))
                    seen.setdefault(DigestCache._key(mv), []).append(j)
                seen[id(m)] = j
            slot[i] = j
        with CACHE._lock:
            CACHE.misses += len(uniq)
        if _gpu_batch_wins(uniq):
            from .. import ops

            ds = ops.sha256_batch(uniq)
        else:  # long messages on the hashing threads, short ones inline (a task costs ~20 us)
            big = [j for j, m in enumerate(uniq) if len(m) >= HOST_THREAD_MIN]
            ds = [None] * len(uniq)
            if len(big) > 1:
                for j, d in zip(big, hash_pool().map(sha256_host, [uniq[j] for j in big])):
                    ds[j] = d
            for j, m in enumerate(uniq):
                if ds[j] is None:
                    ds[j] = sha256_host(m)
        for i in todo:
            out[i] = ds[slot[i]]
            CACHE.put(messages[i], out[i])
    return [_result(d) for d in out]
