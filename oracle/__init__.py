"""CPU oracle for the P2PDL aggregation / digest hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this package, and only as the
checker or the timed CPU baseline -- never as a product code path.  The product
(``p2pdl_amd``) fails loudly when its HIP library is missing; it never falls
back to anything in here.

Two independent restatements live here:

* ``liboracle.so`` (``oracle.c``): scalar C, one element at a time, exactly the
  reference's per-element op order (reference ``aggregator/aggregation.py:15-38``).
* numpy restatements (``*_np``): vectorised over coordinates, same op order.

Parity pinning: FedAvg against golden vectors produced by the reference's own
``aggregate_models`` (``tests/golden/make_golden.py``); SHA-256 against FIPS
180-4 KATs and ``hashlib`` (the function behind ``hashes.SHA256()`` at reference
``utils/crypto.py:56,95``); median / trimmed mean are build-defined
(reference ``README.md:10`` TODO) and cross-checked against
numpy sort and ``torch.median``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

RULE_FEDAVG, RULE_MEDIAN, RULE_TRIMMED = 0, 1, 2


def build(force: bool = False) -> str:
    """Compile oracle.c with gcc (no reference sources involved)."""
    if force or not os.path.exists(_LIB_PATH) or (
        os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "oracle.c"))
    ):
        subprocess.check_call(["make", "-s", "-C", _HERE, "-B" if force else "liboracle.so"])
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        L.oracle_synth_f32.argtypes = [P, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int32,
                                       ctypes.c_float, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]
        L.oracle_synth_f32.restype = None
        L.oracle_fedavg_f32.argtypes = [P, ctypes.c_int32, ctypes.c_int64, P, ctypes.c_float, P]
        L.oracle_fedavg_f32.restype = None
        L.oracle_fedavg_mode_f32.argtypes = [P, ctypes.c_int32, ctypes.c_int64, P, ctypes.c_float, P,
                                             ctypes.c_int32]
        L.oracle_fedavg_mode_f32.restype = None
        L.oracle_robust_f32.argtypes = [P, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32,
                                        ctypes.c_int32, P, ctypes.c_float, P]
        L.oracle_robust_f32.restype = ctypes.c_int
        L.oracle_sha256.argtypes = [P, ctypes.c_uint64, P]
        L.oracle_sha256.restype = None
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def _peer_table(peers):
    arrs = [np.ascontiguousarray(p, dtype=np.float32) for p in peers]
    tbl = (ctypes.c_void_p * len(arrs))(*[_ptr(a) for a in arrs])
    return arrs, tbl


# ---------------------------------------------------------------- synthetic
def synth(n: int, seed: int, peer: int, scale: float, chunk: int = 0, nranks: int = 1,
          rank: int = 0) -> np.ndarray:
    """C restatement of the build's counter PRNG."""
    out = np.empty(n, dtype=np.float32)
    lib().oracle_synth_f32(_ptr(out), n, seed, peer, scale, chunk, nranks, rank)
    return out


def _splitmix64_np(x: np.ndarray) -> np.ndarray:
    x = x + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def synth_np(n: int, seed: int, peer: int, scale: float, chunk: int = 0, nranks: int = 1,
             rank: int = 0) -> np.ndarray:
    """numpy restatement of the same PRNG (independent of the C one)."""
    i = np.arange(n, dtype=np.int64)
    if nranks > 1 and chunk > 0:
        s, j = i // chunk, i % chunk
        i = (s * nranks + rank) * chunk + j
    with np.errstate(over="ignore"):
        u = _splitmix64_np(np.uint64(seed) ^ (np.uint64(peer) << np.uint64(40)) ^ i.astype(np.uint64))
    u = (u >> np.uint64(40)).astype(np.float32)
    x = u * np.float32(2.0 ** -23) - np.float32(1.0)
    return x * np.float32(scale)


def synth_at(idx, seed: int, peer: int, scale: float) -> np.ndarray:
    """The PRNG at arbitrary global coordinates (size-independent checks of
    buffers too large to regenerate on the host)."""
    i = np.asarray(idx, dtype=np.int64)
    with np.errstate(over="ignore"):
        u = _splitmix64_np(np.uint64(seed) ^ (np.uint64(peer) << np.uint64(40)) ^ i.astype(np.uint64))
    u = (u >> np.uint64(40)).astype(np.float32)
    return (u * np.float32(2.0 ** -23) - np.float32(1.0)) * np.float32(scale)


# ---------------------------------------------------------------- FedAvg
def fedavg(peers, w=None, lr: float = 0.1, want_out: bool = False, torch_gpu: bool = False):
    """C restatement of reference aggregator/aggregation.py:15-38.
    torch_gpu: the ops as torch runs them on GPU tensors (acc * fl(1/K) at
    :32; the product's 'fedavg_torch_gpu' rule).

    Returns (w_new, out) where w_new is a new array (input untouched)."""
    arrs, tbl = _peer_table(peers)
    n = arrs[0].size if arrs else 0
    w_new = None if w is None else np.array(w, dtype=np.float32, copy=True)
    out = np.empty(n, dtype=np.float32) if (want_out or w is None) else None
    lib().oracle_fedavg_mode_f32(tbl, len(arrs), n, None if w_new is None else _ptr(w_new),
                                 lr, None if out is None else _ptr(out), int(torch_gpu))
    return w_new, out


def fedavg_np(peers, w=None, lr: float = 0.1, torch_gpu: bool = False):
    """numpy restatement (vectorised over coordinates, same op order).
    Overflow to +-inf and inf - inf = NaN are IEEE results here, as in the
    reference's torch ops (the golden special-value cases): not warned."""
    with np.errstate(over="ignore", invalid="ignore"):
        acc = np.zeros_like(np.asarray(peers[0], dtype=np.float32))
        for p in peers:
            acc = acc + np.asarray(p, dtype=np.float32)
        k = np.float32(len(peers))
        acc = acc * (np.float32(1.0) / k) if torch_gpu else acc / k
        if w is None:
            return None, acc
        return (np.asarray(w, dtype=np.float32) + np.float32(lr) * acc).astype(np.float32), acc


# ------------------------------------------------- 16-bit models (a1-a4)
def to_f32_16(bits, dtype: str) -> np.ndarray:
    """uint16 storage bits of float16 / bfloat16 values -> exact float32."""
    b = np.asarray(bits, dtype=np.uint16)
    if dtype == "float16":
        return b.view(np.float16).astype(np.float32)
    return (b.astype(np.uint32) << np.uint32(16)).view(np.float32)


def round_16(x, dtype: str) -> np.ndarray:
    """float32 -> uint16 bits, round to nearest even, as torch converts
    (c10::Half / c10::BFloat16 from float; a NaN stays a NaN)."""
    x = np.asarray(x, dtype=np.float32)
    if dtype == "float16":
        with np.errstate(over="ignore"):  # out of range -> +-inf, as torch converts
            return x.astype(np.float16).view(np.uint16)
    u = x.view(np.uint32).astype(np.uint64)
    r = ((u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) >> np.uint64(16)).astype(np.uint16)
    return np.where(np.isnan(x), np.uint16(0x7FC0), r).astype(np.uint16)


def round_16_once(x, dtype: str) -> np.ndarray:
    """float64 -> float16 bits with ONE rounding (round to nearest even from
    the exact value): round-to-odd to float32 first (24 >= 11 + 2 bits keeps
    the single rounding exact), then float32 -> float16."""
    assert dtype == "float16"
    x = np.asarray(x, dtype=np.float64)
    f = x.astype(np.float32)
    away = np.abs(f.astype(np.float64)) > np.abs(x)
    f = np.where(away, np.nextafter(f, np.float32(0)), f).astype(np.float32)
    inexact = f.astype(np.float64) != x
    b = f.view(np.uint32) | np.where(inexact & np.isfinite(x), np.uint32(1), np.uint32(0))
    return round_16(b.astype(np.uint32).view(np.float32), dtype)


def fedavg16_np(peers, w, dtype: str, lr: float = 0.1, torch_gpu: bool = False):
    """The reference's ops (aggregation.py:15-38) on a float16 / bfloat16
    model, as torch runs them: every op computed in float32 and rounded to
    the storage type -- acc = +0 (:15); acc = r(acc + u) per update in list
    order (:25-28); acc = r(acc / K) (:31-32; torch_gpu: r(acc * fl(1/K)),
    ATen's division by a CPU scalar on a GPU tensor); t = r(fp32(lr) * acc);
    w = r(w + t) (:36-38).  peers / w / result: uint16 bit arrays."""
    f = lambda b: to_f32_16(b, dtype)
    with np.errstate(over="ignore", invalid="ignore"):  # inf / NaN arithmetic is part of the contract
        acc = np.zeros_like(f(w))
        for p in peers:
            acc = f(round_16(acc + f(p), dtype))
        k = np.float32(len(peers))
        acc = f(round_16(acc * (np.float32(1.0) / k) if torch_gpu else acc / k, dtype))
        t = f(round_16(np.float32(lr) * acc, dtype))
        return round_16(f(w) + t, dtype)


# ---------------------------------------------------------------- robust rules
def trim_count(k: int, trim_frac: float = 0.2) -> int:
    """b = floor(trim_frac * K), computed in exact integers
    for the default 0.2 so K=5*m never lands a hair under an integer."""
    b = int(np.floor(trim_frac * k + 1e-9))
    return b


def robust(peers, rule: int, trim_b: int = 0, w=None, lr: float = 0.1):
    arrs, tbl = _peer_table(peers)
    n = arrs[0].size
    w_new = None if w is None else np.array(w, dtype=np.float32, copy=True)
    out = np.empty(n, dtype=np.float32)
    rc = lib().oracle_robust_f32(tbl, len(arrs), n, rule, trim_b,
                                 None if w_new is None else _ptr(w_new), lr, _ptr(out))
    if rc != 0:
        raise ValueError(f"oracle_robust_f32 rejected K={len(arrs)} rule={rule} b={trim_b}")
    return w_new, out


def f2key_np(x: np.ndarray) -> np.ndarray:
    b = np.asarray(x, dtype=np.float32).view(np.uint32)
    neg = (b & np.uint32(0x80000000)) != 0
    return np.where(neg, ~b, b | np.uint32(0x80000000)).astype(np.uint32)


def key2f_np(k: np.ndarray) -> np.ndarray:
    top = (k & np.uint32(0x80000000)) != 0
    return np.where(top, k & np.uint32(0x7FFFFFFF), ~k).astype(np.uint32).view(np.float32)


def robust_np(peers, rule: int, trim_b: int = 0):
    keys = np.sort(np.stack([f2key_np(p) for p in peers]), axis=0)
    K = keys.shape[0]
    if rule == RULE_MEDIAN:
        return key2f_np(keys[(K - 1) // 2])
    acc = np.zeros(keys.shape[1], dtype=np.float32)
    for r in range(trim_b, K - trim_b):
        acc = acc + key2f_np(keys[r])
    return acc / np.float32(K - 2 * trim_b)


def apply_np(w, agg, lr: float = 0.1):
    return (np.asarray(w, dtype=np.float32) + np.float32(lr) * np.asarray(agg, dtype=np.float32))


# ---------------------------------------------------------------- SHA-256
def sha256(data: bytes) -> bytes:
    buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, dtype=np.uint8)
    out = np.zeros(32, dtype=np.uint8)
    lib().oracle_sha256(_ptr(buf), len(data), _ptr(out))
    return out.tobytes()


def delta_snapshot_np(cur, prev=None):
    """Trainer-side local update, reference node/node.py:272-282: the first
    round (prev None) sends the current state (:275), later rounds
    current - previous (:279, fp32 IEEE subtraction); the new previous is a
    copy of current (:282).  Returns (delta, new_prev)."""
    cur = np.ascontiguousarray(cur, dtype=np.float32)
    if prev is None:
        return cur.copy(), cur.copy()
    return (cur - np.asarray(prev, dtype=np.float32)).astype(np.float32), cur.copy()
