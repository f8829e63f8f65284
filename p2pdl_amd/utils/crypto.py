"""Drop-in for the digest part of reference ``utils/crypto.py``.

The reference signs / verifies with ``ec.ECDSA(hashes.SHA256())``
(utils/crypto.py:54-57 and :92-96): OpenSSL hashes the full serialized update
on every call -- 72 SHA-256 passes over 3 distinct messages per round in the
default configuration.  Here every digest comes from
``utils/digests.py``: each DISTINCT message is hashed once per process (at
arrival by ``DeviceInbox.land(..., digest=True)``, or at its first sign /
verify), later calls on the same object -- or on equal bytes -- reuse it, and
the EC step signs / verifies the 32-byte digest with
``Prehashed(SHA256())`` -- byte-compatible with the reference's signatures
because ECDSA signs the digest.  Single messages hash on the host (SHA-NI);
batches of many distinct messages go to the gfx950 batch kernel
(``p2p_sha256_batch``; boundary in DESIGN.md §3 K3).  The EC arithmetic (out
of scope) needs the ``cryptography`` package; it is imported lazily and is
absent from this build image, so the EC half is "parity unpinned" here
(DESIGN.md).

Function names, arguments and the never-raise / return-False behaviour of
``verify_signature`` mirror the reference (:64-101): a maintainer points
``p2pdl/utils/crypto.py`` at this module and ``utils/broadcast.py`` (which
imports sign_data / verify_signature from it, :4) is left untouched.
"""
from __future__ import annotations

import logging
import pickle
from typing import Iterable, Sequence

from . import digests


# what `from p2pdl.utils.crypto import ...` finds in the reference
# (node/node.py:16, main.py:7, utils/broadcast.py:4), plus the batched forms
__all__ = ["KeyServer", "generate_key_pair", "sign_data", "verify_signature", "verify_signature_2",
           "verify_signatures_batch", "digest_updates"]


class KeyServer:
    """In-process public key registry (reference utils/crypto.py:7-40)."""

    def __init__(self):
        self.public_key_store = {}

    def register_key(self, addr, port, public_key):
        node_id = (addr, port)
        if node_id not in self.public_key_store:
            self.public_key_store[node_id] = public_key
        else:
            logging.warning(f"Public key already exists for {addr}:{port}")

    def get_key(self, addr, port):
        key = self.public_key_store.get((addr, port))
        if not key:
            logging.warning(f"Public key not found for {addr}:{port}")
        return key

    def get_all_keys(self):
        return self.public_key_store


def _ec():
    """The EC half (out of scope, host): the `cryptography` package.  A
    missing package raises ImportError -- the reference fails the same way,
    at import (utils/crypto.py:1-3) -- it is never reported as a bad
    signature."""
    try:
        from cryptography.hazmat.primitives import hashes
        from cryptography.hazmat.primitives.asymmetric import ec
        from cryptography.hazmat.primitives.asymmetric import utils as asym_utils
    except ImportError as e:
        raise ImportError("p2pdl_amd.utils.crypto: the EC step needs the 'cryptography' package") from e
    return hashes, ec, asym_utils


def digest_updates(messages: Sequence[bytes]) -> list[bytes]:
    """SHA-256 of every message; a message that occurs several times -- or
    was hashed before -- is hashed once (node/node.py:155,187-206 hash the
    same 3 updates 72 times per round).  Many distinct messages go to the
    GPU batch kernel in one launch (``digests.digest_many``)."""
    return digests.digest_many(messages)


def generate_key_pair():
    """ECDSA key pair on SECP256R1 (reference :42-48)."""
    _, ec, _ = _ec()
    private_key = ec.generate_private_key(ec.SECP256R1())
    return private_key, private_key.public_key()


def sign_data(private_key, data, digest: bytes | None = None):
    """ECDSA(SHA-256(data)) like reference :50-59 -- the SHA-256 from the
    digest cache (hashed once per distinct message), the EC step on the
    32-byte digest (Prehashed), which yields the same signatures as
    ECDSA(SHA256()) over the data.  ``data`` may also be a PinnedMessage
    window (node/inbox.py) -- the serialized update where it arrived."""
    hashes, ec, asym_utils = _ec()
    if digest is None:
        if not isinstance(data, (bytes, bytearray, memoryview)) and not digests._is_window(data):
            raise TypeError(f"data must be bytes-like, got {type(data).__name__}")  # as cryptography's sign
        digest = digests.digest_of(data)
    return private_key.sign(digest, ec.ECDSA(asym_utils.Prehashed(hashes.SHA256())))


def verify_signature_2(key_server, addr, port, data, signature):
    """Reference :61-62 (imported by node/node.py:16): accepts everything."""
    return True


def verify_signature(key_server, addr, port, data, signature, digest: bytes | None = None) -> bool:
    """Reference :64-101: False on a missing key (:71-80), None data
    (:83-85), a serialisation failure (:87-92) or a bad signature (:94-101).
    ``digest`` (optional) is SHA-256(data) computed earlier, e.g. by
    ``verify_signatures_batch``.  A missing GPU or `cryptography` raises."""
    hashes, ec, asym_utils = _ec()
    public_key = key_server.get_key(addr, port)
    if not public_key:
        logging.error(f"Public key for {addr}:{port} not found.")
        return False
    if digest is None:
        if data is None:
            logging.error(f"Cannot verify signature: data is None for {addr}:{port}")
            return False
        if not isinstance(data, bytes) and not digests._is_window(data):
            try:
                data = pickle.dumps(data)
            except Exception as e:
                logging.error(f"Failed to serialize data for {addr}:{port}: {e}")
                return False
        digest = digests.digest_of(data)
    try:
        public_key.verify(signature, digest, ec.ECDSA(asym_utils.Prehashed(hashes.SHA256())))
        return True
    except Exception as e:  # reference returns False on any verification failure
        logging.error(f"Signature verification failed for {addr}:{port}: {e}")
        return False


def verify_signatures_batch(key_server, items: Iterable[tuple]) -> list[bool]:
    """verify_signature over many (addr, port, data, signature) items with
    every distinct data blob hashed once (the tester's ready handler verifies
    the same bytes once per signature, node/node.py:187-206); many distinct
    blobs go to the GPU batch kernel in one launch.  Per-item results follow
    verify_signature."""
    _ec()
    items = list(items)
    blobs, ok = [], []
    for addr, port, data, _ in items:
        if data is None:
            blobs.append(None)
            continue
        try:
            blobs.append(data if isinstance(data, bytes) or digests._is_window(data) else pickle.dumps(data))
        except Exception as e:
            logging.error(f"Failed to serialize data for {addr}:{port}: {e}")
            blobs.append(None)
    live = [b for b in blobs if b is not None]
    found = iter(digest_updates(live))
    for (addr, port, data, sig), b in zip(items, blobs):
        if b is None:
            if data is None:
                logging.error(f"Cannot verify signature: data is None for {addr}:{port}")
            ok.append(False)
            continue
        ok.append(verify_signature(key_server, addr, port, None, sig, digest=next(found)))
    return ok
