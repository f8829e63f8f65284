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

from p2pdl_amd.utils import crypto


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
    launches = []

    def sha256_batch(msgs, device=None):  # hashlib in place of the GPU launch (CPU test)
        launches.append(list(msgs))
        return [hashlib.sha256(m).digest() for m in msgs]

    monkeypatch.setattr(crypto, "_ec", fake_ec)
    monkeypatch.setattr(crypto.ops, "sha256_batch", sha256_batch)
    ks = crypto.KeyServer()
    pub = FakePublicKey()
    ks.register_key("127.0.0.1", 7001, pub)
    return types.SimpleNamespace(ks=ks, pub=pub, priv=FakePrivateKey(), launches=launches)


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


def test_72_hashes_become_3_in_one_launch(env):
    """Default round: 3 distinct updates, 4 testers x 3 readies x
    4 signatures + echo verifies = 72 hash passes in the reference."""
    updates = [pickle.dumps({"trainer": t, "w": bytes(range(256)) * (t + 1)}) for t in range(3)]
    sigs = {u: crypto.sign_data(env.priv, u) for u in updates}
    env.launches.clear()
    items = [("127.0.0.1", 7001, u, sigs[u]) for _ in range(24) for u in updates]
    assert len(items) == 72
    assert crypto.verify_signatures_batch(env.ks, items) == [True] * 72
    assert len(env.launches) == 1 and sorted(env.launches[0]) == sorted(updates)
    assert env.pub.calls == 72  # the EC check still runs per signature


def test_batch_mixed_results(env):
    good = b"m1"
    items = [("127.0.0.1", 7001, good, crypto.sign_data(env.priv, good)),
             ("127.0.0.1", 7001, good, b"forged"),
             ("10.0.0.9", 9, good, b"x"),
             ("127.0.0.1", 7001, None, b"x"),
             ("127.0.0.1", 7001, lambda: 0, b"x")]
    env.launches.clear()
    assert crypto.verify_signatures_batch(env.ks, items) == [True, False, False, False, False]
    assert env.launches == [[good]]


def test_digest_updates_dedupes_and_keeps_order(env):
    msgs = [b"b", b"a", b"b", bytearray(b"a"), b""]
    got = crypto.digest_updates(msgs)
    assert got == [hashlib.sha256(bytes(m)).digest() for m in msgs]
    assert env.launches == [[b"b", b"a", b""]]


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
    """The real HIP batch kernel behind digest_updates: 72 items, 3 distinct."""
    calls = []
    real = crypto.ops.sha256_batch
    monkeypatch.setattr(crypto.ops, "sha256_batch", lambda m, device=None: calls.append(len(m)) or real(m, device))
    updates = [pickle.dumps({"t": t, "w": bytes(range(256)) * (1000 + 37 * t)}) for t in range(3)]
    msgs = [u for _ in range(24) for u in updates]
    assert crypto.digest_updates(msgs) == [hashlib.sha256(m).digest() for m in msgs]
    assert calls == [3]
