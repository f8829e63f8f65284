"""ctypes binding of libp2pdl_hip.so (the C ABI in include/p2pdl.h).

This is the ONLY route to the hot path: there is no CPU or eager-torch
fallback.  If the library is missing or no ROCm device is visible, every op
raises ``NativeUnavailable`` -- loudly, by design.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# P2P_LIB selects a diagnostic build (csrc/Makefile `diag`); default: the product library
LIB_PATH = os.environ.get("P2P_LIB") or os.path.join(_HERE, "libp2pdl_hip.so")
ABI_VERSION = 9  # include/p2pdl.h P2P_ABI_VERSION

P2P_RULE_FEDAVG, P2P_RULE_MEDIAN, P2P_RULE_TRIMMED, P2P_RULE_FEDAVG_TORCH_GPU = 0, 1, 2, 3
P2P_DTYPE_F16, P2P_DTYPE_BF16 = 1, 2
P2P_HINT_SHARE_CUS = 1  # include/p2pdl.h (ABI 9)

# Every symbol include/p2pdl.h declares (tests check the .so exports them).
EXPORTS = (
    "p2p_abi_version", "p2p_strerror", "p2p_tile_elems",
    "p2p_fedavg_apply_f32", "p2p_mean_f32", "p2p_fedavg_apply_devk_f32", "p2p_fedavg_apply_16",
    "p2p_median_f32", "p2p_trimmed_mean_f32", "p2p_aggregate_f32", "p2p_aggregate_ex_f32",
    "p2p_aggregate_segments_f32", "p2p_fedavg_split_plan", "p2p_fedavg_split_segments_f32",
    "p2p_fedavg_split_rows_f32", "p2p_fedavg_split_chunks_f32", "p2p_apply_f32",
    "p2p_sha256_batch", "p2p_digest_accept", "p2p_fill_synthetic_f32",
    "p2p_delta_snapshot_f32", "p2p_delta_snapshot_segments_f32", "p2p_land_segments_f32",
)


class NativeUnavailable(RuntimeError):
    """The HIP library or a ROCm device is missing: the hot path cannot run."""


class P2PError(RuntimeError):
    """A non-zero status from the C ABI."""


def host_extension(name: str):
    """A CPython extension built beside the HIP library by csrc/Makefile
    (``_host_tables``: the drop-in's peer-table gather; ``_wire``: the
    restricted pickle machine of the receive path).  The product imports
    them unconditionally: a build that failed to produce one fails here,
    loudly, instead of running a slower pure-Python path."""
    import importlib

    try:
        return importlib.import_module(f"p2pdl_amd.{name}")
    except ImportError as e:
        raise NativeUnavailable(f"p2pdl_amd.{name} is not built ({e}); run `make -C p2pdl_amd/csrc` "
                                "or __graft_entry__.build()") from e


_lib = None
_lock = threading.Lock()
_cuda_ok = False  # a ROCm device was seen (checked once)

_P = ctypes.c_void_p
_I32, _I64, _U64, _F32 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float

_SIGS = {
    "p2p_abi_version": ([], _I32),
    "p2p_strerror": ([_I32], ctypes.c_char_p),
    "p2p_tile_elems": ([_I32, _I32], _I64),
    "p2p_fedavg_apply_f32": ([_P, _I32, _I64, _P, _F32, _P], _I32),
    "p2p_mean_f32": ([_P, _I32, _I64, _P, _P], _I32),
    "p2p_fedavg_apply_devk_f32": ([_P, _P, _I32, _I64, _P, _F32, _P, _P], _I32),
    "p2p_fedavg_apply_16": ([_P, _I32, _I64, _P, _F32, _I32, _I32, _P], _I32),
    "p2p_median_f32": ([_P, _I32, _I64, _P, _P], _I32),
    "p2p_trimmed_mean_f32": ([_P, _I32, _I64, _I32, _P, _P], _I32),
    "p2p_aggregate_f32": ([_P, _I32, _I64, _I32, _I32, _F32, _P, _P, _P], _I32),
    "p2p_aggregate_ex_f32": ([_P, _I32, _I64, _I32, _I32, _F32, _P, _P, _I32, _P], _I32),
    "p2p_aggregate_segments_f32": ([_P, _I32, _I64, _I32, _I32, _I32, _F32, _P], _I32),
    "p2p_fedavg_split_plan": ([_I32, _I64], _I64),
    "p2p_fedavg_split_segments_f32": ([_P, _I64, _P, _I32, _I32, _F32, _P], _I32),
    "p2p_fedavg_split_rows_f32": ([_P, _I32, _I64, _P, _I32, _F32, _P], _I32),
    "p2p_fedavg_split_chunks_f32": ([_P, _I64, _P, _I32, _I32, _F32, _P], _I32),
    "p2p_apply_f32": ([_P, _P, _F32, _I64, _P], _I32),
    "p2p_sha256_batch": ([_P, _P, _I32, _P, _P], _I32),
    "p2p_digest_accept": ([_P, _P, _P, _I32, _P, _P, _P], _I32),
    "p2p_fill_synthetic_f32": ([_P, _I64, _U64, _I32, _F32, _I64, _I32, _I32, _P], _I32),
    "p2p_delta_snapshot_f32": ([_P, _P, _P, _I64, _I32, _P], _I32),
    "p2p_delta_snapshot_segments_f32": ([_P, _I32, _I64, _I32, _P], _I32),
    "p2p_land_segments_f32": ([_P, _U64, _P, _I32, _I64, _P], _I32),
}


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """dlopen the library and bind every ABI symbol (no GPU needed)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise NativeUnavailable(
                f"p2pdl_amd: {path} is missing -- build it with `make -C p2pdl_amd/csrc` "
                "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
        lib = ctypes.CDLL(path)
        for name, (args, res) in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        got = lib.p2p_abi_version()
        if got != ABI_VERSION:
            raise NativeUnavailable(f"p2pdl_amd: ABI version {got} != expected {ABI_VERSION}")
        _lib = lib
        return lib


def lib() -> ctypes.CDLL:
    return _lib if _lib is not None else load_library()


def require_device(t) -> None:
    """The hot path runs only on a ROCm device; CPU tensors are rejected."""
    import torch

    global _cuda_ok
    if not _cuda_ok:
        _cuda_ok = torch.cuda.is_available()
    if not _cuda_ok:
        raise NativeUnavailable("p2pdl_amd: no ROCm GPU visible; the HIP hot path cannot run "
                                "(there is no CPU fallback)")
    if t.device.type != "cuda":
        raise RuntimeError(f"p2pdl_amd: tensors must be on a ROCm device, got {t.device}")


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().p2p_strerror(rc)
        raise P2PError(f"{what} failed ({rc}): {msg.decode() if msg else 'unknown'}")


def stream_handle(device=None) -> int:
    """The raw hipStream_t of the current stream of ``device`` (default: the
    current device) -- what torch.cuda.current_stream(device).cuda_stream
    returns, without building the Stream object (a few us per launch at the
    reference's MLP size, where the whole call is host-bound)."""
    import torch

    if device is None:
        idx = torch.cuda.current_device()
    elif isinstance(device, int):
        idx = device
    else:
        idx = device.index if device.index is not None else torch.cuda.current_device()
    return torch._C._cuda_getCurrentRawStream(idx)
