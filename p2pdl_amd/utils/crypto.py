"""Drop-in for the digest part of reference ``utils/crypto.py``.

The reference signs / verifies with ``ec.ECDSA(hashes.SHA256())``
(utils/crypto.py:54-57 and :92-96): OpenSSL hashes the full serialized update
on every call -- 72 SHA-256 passes over 3 distinct messages per round in the
default configuration.  Here the SHA-256 runs in the gfx950
batch kernel (``p2p_sha256_batch``), once per DISTINCT message, and the EC
step signs / verifies the 32-byte digest with ``Prehashed(SHA256())`` --
byte-compatible with the reference's signatures because ECDSA signs the
digest.  The EC arithmetic (out of scope) needs the ``cryptography`` package;
it is imported lazily and is absent from this build image, so the EC half is
"parity unpinned" here.

Function names, arguments and the never-raise / return-False behaviour of
``verify_signature`` mirror the reference (:64-101).
"""
from __future__ import annotations

import logging
import pickle
from typing import Iterable, Sequence

from .. import ops


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
    try:
        from cryptography.hazmat.primitives import hashes
        from cryptography.hazmat.primitives.asymmetric import ec
        from cryptography.hazmat.primitives.asymmetric import utils as asym_utils
    except ImportError as e:  # same failure the reference has without the package
        raise ImportError("p2pdl_amd.utils.crypto: the EC step needs the 'cryptography' package") from e
    return hashes, ec, asym_utils


def _as_bytes(data) -> bytes:
    return data if isinstance(data, bytes) else pickle.dumps(data)  # reference :82-88


def digest_updates(messages: Sequence[bytes]) -> list[bytes]:
    """SHA-256 of every message in one GPU launch (duplicates hashed once)."""
    uniq, index = [], {}
    for m in messages:
        if m not in index:
            index[m] = len(uniq)
            uniq.append(m)
    d = ops.sha256_batch(uniq) if uniq else []
    return [d[index[m]] for m in messages]


def generate_key_pair():
    """ECDSA key pair on SECP256R1 (reference :42-48)."""
    _, ec, _ = _ec()
    private_key = ec.generate_private_key(ec.SECP256R1())
    return private_key, private_key.public_key()


def sign_data(private_key, data, digest: bytes | None = None):
    """ECDSA(SHA-256(data)) like reference :50-59, digest computed on the GPU."""
    hashes, ec, asym_utils = _ec()
    digest = digest if digest is not None else digest_updates([_as_bytes(data)])[0]
    return private_key.sign(digest, ec.ECDSA(asym_utils.Prehashed(hashes.SHA256())))


def verify_signature(key_server, addr, port, data, signature, digest: bytes | None = None) -> bool:
    """Reference :64-101 semantics: False on a missing key, None data, a
    serialisation failure or a bad signature; never raises."""
    public_key = key_server.get_key(addr, port)
    if not public_key:
        logging.error(f"Public key for {addr}:{port} not found.")
        return False
    if data is None and digest is None:
        logging.error(f"Cannot verify signature: data is None for {addr}:{port}")
        return False
    try:
        hashes, ec, asym_utils = _ec()
        if digest is None:
            digest = digest_updates([_as_bytes(data)])[0]
        public_key.verify(signature, digest, ec.ECDSA(asym_utils.Prehashed(hashes.SHA256())))
        return True
    except Exception as e:  # reference returns False on any failure
        logging.error(f"Signature verification failed for {addr}:{port}: {e}")
        return False


def verify_signatures_batch(key_server, items: Iterable[tuple]) -> list[bool]:
    """Verify many (addr, port, data, signature) at once: every distinct data
    blob is hashed once in one GPU launch (node/node.py:187-206 verifies the
    same bytes once per signature)."""
    items = list(items)
    blobs = [_as_bytes(d) for _, _, d, _ in items]
    digests = digest_updates(blobs)
    return [verify_signature(key_server, a, p, None, s, digest=g)
            for (a, p, _, s), g in zip(items, digests)]
