"""Digest / verify drop-in (p2pdl_amd.utils.crypto) vs reference utils/crypto.py:50-101.

The EC step needs the `cryptography` package, which is absent from this image
(SURVEY.md §8(c)): ECDSA itself is "parity unpinned".  What is pinned here is
everything around it, with fake key objects exposing the same .sign/.verify
calls: the never-raise / return-False contract of verify_signature
(reference :64-101), the pickling of non-bytes data (:82-88), the dedupe of
the 72 hashes per round into one launch over the distinct messages
(node/node.py:155,187-206), and that a missing `cryptography` raises instead
of reading as a bad signature.  CPU tests replace the GPU digest with
hashlib (the function behind hashes.SHA256()); the -m gpu test runs the HIP
kernel.
"""
import hashlib
import pickle
import types

import pytest

from p2pdl_amd import ops
from p2pdl_amd.utils import crypto, digests


class FakeAlg:
    def __init__(self, inner):
        self.inner = inner


def fake_ec():
    """Stand-ins for cryptography's hashes / ec / asym_utils modules."""
    hashes = types.SimpleNamespace(SHA256=lambda: "sha256")
    ec = types.SimpleNamespace(ECDSA=FakeAlg)
    asym = types.SimpleNamespace(Prehashed=lambda h: ("prehashed", h))
    return hashes, ec, asym


class BadSignature(Exception):
    pass


class FakePrivateKey:
    def sign(self, digest, alg):
        assert alg.inner == ("prehashed", "sha256") and len(digest) == 32
        return b"sig:" + digest


class FakePublicKey:
    def __init__(self):
        self.calls = 0

    def verify(self, signature, digest, alg):
        self.calls += 1
        assert alg.inner == ("prehashed", "sha256")
        if signature != b"sig:" + digest:
            raise BadSignature("bad signature")


@pytest.fixture
def env(monkeypatch):
    launches, hashed = [], []

    def sha256_batch(msgs, device=None):  # hashlib in place of the GPU launch (CPU test)
        launches.append(list(msgs))
        return [hashlib.sha256(m).digest() for m in msgs]

    real_host = digests.sha256_host

    def sha256_host(data):
        hashed.append(bytes(digests._buffer(data)))
        return real_host(data)

    monkeypatch.setattr(crypto, "_ec", fake_ec)
    monkeypatch.setattr(ops, "sha256_batch", sha256_batch)
    monkeypatch.setattr(digests, "sha256_host", sha256_host)
    digests.CACHE.clear()
    ks = crypto.KeyServer()
    pub = FakePublicKey()
    ks.register_key("127.0.0.1", 7001, pub)
    yield types.SimpleNamespace(ks=ks, pub=pub, priv=FakePrivateKey(), launches=launches, hashed=hashed)
    digests.CACHE.clear()


def test_sign_then_verify_roundtrip(env):
    data = pickle.dumps({"w": list(range(100))})
    sig = crypto.sign_data(env.priv, data)
    assert sig == b"sig:" + hashlib.sha256(data).digest()  # ECDSA over SHA-256(data), prehashed
    assert crypto.verify_signature(env.ks, "127.0.0.1", 7001, data, sig) is True


def test_verify_never_raises_and_returns_false(env, caplog):
    data = b"update-bytes"
    sig = crypto.sign_data(env.priv, data)
    # wrong signature / wrong data -> False (reference :97-101)
    assert crypto.verify_signature(env.ks, "127.0.0.1", 7001, data, b"sig:" + bytes(32)) is False
    assert crypto.verify_signature(env.ks, "127.0.0.1", 7001, data + b"!", sig) is False
    # unknown sender -> False before any hashing (reference :71-80)
    n = len(env.launches)
    assert crypto.verify_signature(env.ks, "10.0.0.1", 1, data, sig) is False
    # None data -> False (reference :83-85)
    assert crypto.verify_signature(env.ks, "127.0.0.1", 7001, None, sig) is False
    assert len(env.launches) == n
    # data that cannot be pickled -> False (reference :87-92)
    assert crypto.verify_signature(env.ks, "127.0.0.1", 7001, lambda: 0, sig) is False
    assert "verification failed" in caplog.text and "not found" in caplog.text


def test_non_bytes_data_is_pickled_like_the_reference(env):
    obj = {"a": [1, 2, 3]}
    sig = crypto.sign_data(env.priv, pickle.dumps(obj))
    assert crypto.verify_signature(env.ks, "127.0.0.1", 7001, obj, sig) is True  # :82-88
    with pytest.raises(TypeError):  # sign_data passes data to ECDSA as is (:54-57)
        crypto.sign_data(env.priv, obj)


def test_72_hashes_become_3(env):
    """Default round: 3 distinct updates, 4 testers x 3 readies x
    4 signatures + echo verifies = 72 hash passes in the reference."""
    updates = [pickle.dumps({"trainer": t, "w": bytes(range(256)) * (t + 1)}) for t in range(3)]
    sigs = {u: crypto.sign_data(env.priv, u) for u in updates}
    items = [("127.0.0.1", 7001, u, sigs[u]) for _ in range(24) for u in updates]
    assert len(items) == 72
    assert crypto.verify_signatures_batch(env.ks, items) == [True] * 72
    assert sorted(env.hashed) == sorted(updates) and env.launches == []  # 3 host hashes, no launch
    assert env.pub.calls == 72  # the EC check still runs per signature


def test_reference_round_with_reference_call_signatures(env):
    """The reference's own per-round calls, unchanged (node/node.py:145 ->
    utils/broadcast.py:14, :155, :202), on the objects the reference holds:
    each tester's copy of an update comes out of its own pickle.loads of the
    envelope (:112), the ready message carries yet another copy (:175).
    Each distinct update is hashed once; every other call is a cache hit by
    identity or by content."""
    updates = [pickle.dumps({"trainer": t, "w": bytes(range(256)) * (50 + t)}) for t in range(3)]
    testers = 4
    copies = [[pickle.loads(pickle.dumps({"model": u}))["model"] for u in updates] for _ in range(testers)]
    sig = {}
    for i in range(testers):  # 12 echo signs over each tester's own copy
        for t in range(3):
            sig[i, t] = crypto.sign_data(env.priv, copies[i][t])
    for t in range(3):  # 12 echo verifies over the trainer's own local_update (:155)
        for i in range(testers):
            assert crypto.verify_signature(env.ks, "127.0.0.1", 7001, updates[t], sig[i, t])
    for i in range(testers):  # 48 ready verifies: per ready message, its own copy (:175, :202)
        for t in range(3):
            ready_copy = pickle.loads(pickle.dumps({"local_update": updates[t]}))["local_update"]
            for j in range(testers):
                assert crypto.verify_signature(env.ks, "127.0.0.1", 7001, ready_copy, sig[j, t])
    assert env.pub.calls == 60 and len(env.hashed) == 3
    assert digests.CACHE.hits_content >= 3 and digests.CACHE.hits_identity >= 40


def test_many_distinct_messages_take_the_gpu_batch(env, monkeypatch):
    monkeypatch.setattr(digests, "GPU_BATCH_MIN", 3)
    msgs = [b"b", b"a", b"b", bytearray(b"a"), b"", b"c"]
    got = crypto.digest_updates(msgs)
    assert got == [hashlib.sha256(bytes(m)).digest() for m in msgs]
    assert env.launches == [[b"b", b"a", b"", b"c"]] and env.hashed == []
    env.launches.clear()
    assert crypto.digest_updates(msgs) == got and env.launches == []  # all cached now


def test_batch_mixed_results(env):
    good = b"m1"
    items = [("127.0.0.1", 7001, good, crypto.sign_data(env.priv, good)),
             ("127.0.0.1", 7001, good, b"forged"),
             ("10.0.0.9", 9, good, b"x"),
             ("127.0.0.1", 7001, None, b"x"),
             ("127.0.0.1", 7001, lambda: 0, b"x")]
    env.hashed.clear()
    assert crypto.verify_signatures_batch(env.ks, items) == [True, False, False, False, False]
    assert env.hashed == []  # signed above: cached


def test_digest_updates_dedupes_and_keeps_order(env):
    msgs = [b"b", b"a", b"b", bytearray(b"a"), b""]
    got = crypto.digest_updates(msgs)
    assert got == [hashlib.sha256(bytes(m)).digest() for m in msgs]
    assert sorted(env.hashed) == [b"", b"a", b"b"] and env.launches == []


def test_cache_content_hit_needs_equal_bytes(env):
    """Same length, head and tail but one byte different in the middle: a
    miss (the memcmp decides), with the right digest."""
    a = bytes(100) + b"x" + bytes(100)
    b = bytes(100) + b"y" + bytes(100)
    assert digests.digest_of(a) == hashlib.sha256(a).digest()
    assert digests.digest_of(b) == hashlib.sha256(b).digest()
    assert digests.digest_of(bytearray(b)) == hashlib.sha256(b).digest()
    assert len(env.hashed) == 2


def test_cache_is_bounded(env):
    cache = digests.DigestCache(max_entries=4, max_bytes=1000)
    msgs = [bytes([i]) * 300 for i in range(6)]
    for m in msgs:
        cache.put(m, hashlib.sha256(m).digest())
    assert len(cache) <= 3 and cache._held <= 1000
    assert cache.get(msgs[-1]) == hashlib.sha256(msgs[-1]).digest()
    assert cache.get(msgs[0]) is None  # least recently used went first
    cache.put(bytearray(b"mutable"), bytes(32))  # never kept
    assert cache.get(b"mutable") is None


def test_missing_cryptography_raises_importerror(monkeypatch):
    """ADVICE/VERDICT r01: without `cryptography` every verify used to log
    "verification failed" and return False; the reference fails loudly at
    import (utils/crypto.py:1-3)."""
    import builtins

    real_import = builtins.__import__

    def no_cryptography(name, *a, **k):
        if name.startswith("cryptography"):
            raise ImportError("No module named 'cryptography'")
        return real_import(name, *a, **k)

    monkeypatch.setattr(builtins, "__import__", no_cryptography)
    ks = crypto.KeyServer()
    ks.register_key("a", 1, FakePublicKey())
    with pytest.raises(ImportError):
        crypto.verify_signature(ks, "a", 1, b"x", b"sig")
    with pytest.raises(ImportError):
        crypto.sign_data(FakePrivateKey(), b"x")
    with pytest.raises(ImportError):
        crypto.verify_signatures_batch(ks, [("a", 1, b"x", b"s")])


def test_key_server_semantics(caplog):
    ks = crypto.KeyServer()
    ks.register_key("a", 1, "k1")
    ks.register_key("a", 1, "k2")  # reference keeps the first and warns
    assert ks.get_key("a", 1) == "k1" and "already exists" in caplog.text
    assert ks.get_key("b", 2) is None and "not found" in caplog.text
    assert ks.get_all_keys() == {("a", 1): "k1"}


@pytest.mark.gpu
def test_gpu_digests_match_hashlib_with_dedupe(cuda, monkeypatch):
    """The real HIP batch kernel behind digest_updates (the GPU boundary set
    low): 72 items, 3 distinct, one launch over the 3."""
    calls = []
    real = ops.sha256_batch
    monkeypatch.setattr(ops, "sha256_batch", lambda m, device=None: calls.append(len(m)) or real(m, device))
    monkeypatch.setattr(digests, "GPU_BATCH_MIN", 2)
    monkeypatch.setattr(digests, "GPU_MAX_MESSAGE", 1 << 30)
    digests.CACHE.clear()
    updates = [pickle.dumps({"t": t, "w": bytes(range(256)) * (1000 + 37 * t)}) for t in range(3)]
    msgs = [u for _ in range(24) for u in updates]
    assert crypto.digest_updates(msgs) == [hashlib.sha256(m).digest() for m in msgs]
    assert calls == [3]
    digests.CACHE.clear()


def test_module_exports_what_the_reference_imports():
    """node/node.py:16, main.py:7 and utils/broadcast.py:4 import these names
    from p2pdl.utils.crypto; a star import of the drop-in provides them."""
    ns = {}
    exec("from p2pdl_amd.utils.crypto import *", ns)
    for name in ("KeyServer", "generate_key_pair", "verify_signature", "verify_signature_2", "sign_data"):
        assert name in ns, name
    assert ns["verify_signature_2"](None, "a", 1, b"x", b"s") is True  # reference :61-62


def test_bench_digest_flow_record_on_cpu():
    """bench.py's digest_flow record (the reference's per-round 72 sign /
    verify digests over 3 MLP updates) runs on the host: the
    product hashes 3 times and every signature is over hashlib's digest."""
    import bench

    rec = bench.run_digest_flow(None, 1)
    cfg = rec["config"]
    assert cfg["hashes_product"] == 3 and cfg["hashes_reference"] == 72
    assert cfg["message_bytes"] > 2_000_000 and rec["ms_per_step"] > 0
    assert len(digests.CACHE) == 0  # the record leaves the process cache empty
