"""Tensor-level entry points to the gfx950 kernels (via the C ABI).

All functions take torch tensors that already live on a ROCm device, launch
on ``torch.cuda.current_stream()`` and return without synchronising (except
where a host result is requested, e.g. ``sha256_batch`` returning bytes).
Peer tensors are never stacked or copied: the kernels read them through a
device-resident table of K base pointers (SURVEY.md §8(b) "Ownership").
"""
from __future__ import annotations

import math
import threading
from collections import OrderedDict
from typing import Iterable, Sequence

import numpy as np
import torch

from . import _native as N
from ._native import P2P_RULE_FEDAVG, P2P_RULE_FEDAVG_TORCH_GPU, P2P_RULE_MEDIAN, P2P_RULE_TRIMMED

# the chunk list's C fill (csrc/host_tables.cpp); no silent fallback when it is not built
_host_tables = N.host_extension("_host_tables")

# 'fedavg': the reference's ops as torch runs them on CPU tensors (true
# division by K; the golden vectors).  'fedavg_torch_gpu': the same ops as
# torch runs them on GPU tensors -- the reference's deployment, model on cuda
# (node/node.py:28-29) -- where `acc /= K` is acc * fl(1/K) (include/p2pdl.h).
RULES = {"fedavg": P2P_RULE_FEDAVG, "mean": P2P_RULE_FEDAVG, "median": P2P_RULE_MEDIAN,
         "trimmed": P2P_RULE_TRIMMED, "trimmed_mean": P2P_RULE_TRIMMED,
         "fedavg_torch_gpu": P2P_RULE_FEDAVG_TORCH_GPU}
FEDAVG_RULES = (P2P_RULE_FEDAVG, P2P_RULE_FEDAVG_TORCH_GPU)
MAX_ROBUST_PEERS = 256
DEFAULT_TRIM_FRAC = 0.2


def rule_id(rule) -> int:
    if isinstance(rule, int):
        if rule not in (0, 1, 2, 3):
            raise ValueError(f"unknown aggregation rule id {rule}")
        return rule
    try:
        return RULES[str(rule).lower()]
    except KeyError:
        raise ValueError(f"unknown aggregation rule {rule!r}; expected one of {sorted(RULES)}") from None


def trim_count(k: int, trim_frac: float = DEFAULT_TRIM_FRAC) -> int:
    """b = floor(trim_frac * K); the epsilon keeps exact
    products such as 0.2*5 from landing one ulp under an integer."""
    b = int(math.floor(trim_frac * k + 1e-9))
    if b < 0 or k - 2 * b < 1:
        raise ValueError(f"trim_frac={trim_frac} leaves no ranks for K={k}")
    return b


def _check_f32(t: torch.Tensor, name: str, device) -> None:
    if t.dtype != torch.float32:
        raise TypeError(f"{name}: expected float32, got {t.dtype}")
    if t.device != device:
        raise RuntimeError(f"{name}: expected all tensors on {device}, got {t.device}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")


def pointer_table(tensors: Sequence[torch.Tensor], device) -> torch.Tensor:
    """Device int64 tensor of data pointers (one small non-blocking H2D copy
    through the pinned staging ring).  It remembers the shortest tensor it
    points into, so a call over more elements than that raises instead of
    reading past a peer buffer (``table_covers``)."""
    host = np.array([t.data_ptr() for t in tensors], dtype=np.int64)
    table = _RING.to_device(host, device).view(torch.int64)
    table._p2p_min_numel = min((t.numel() for t in tensors), default=0)
    return table


def table_covers(table: torch.Tensor, n: int, what: str = "table") -> None:
    """A prebuilt pointer table must point into buffers of >= n elements
    (checked when pointer_table built it; a table from elsewhere is the
    caller's contract)."""
    m = getattr(table, "_p2p_min_numel", None)
    if m is not None and n > m:
        raise ValueError(f"{what} points into buffers of {m} elements; the call covers {n}")


def _peer_inputs(peers: Sequence[torch.Tensor], n: int, device):
    if len(peers) == 0:
        raise ValueError("need at least one peer update")
    for i, p in enumerate(peers):
        _check_f32(p, f"peers[{i}]", device)
        if p.numel() != n:
            raise ValueError(f"peers[{i}] has {p.numel()} elements, expected {n}")
    return pointer_table(peers, device)


# ------------------------------------------------------------------ K1 / K2
def aggregate(peers: Sequence[torch.Tensor], rule="fedavg", *, w: torch.Tensor | None = None,
              out: torch.Tensor | None = None, lr: float = 0.1, trim_b: int | None = None,
              trim_frac: float = DEFAULT_TRIM_FRAC, table: torch.Tensor | None = None,
              share_cus: bool = False) -> None:
    """One flat buffer: out = rule(peers); w += lr * out (when w is given).

    ``table`` may pass a prebuilt device pointer table (benchmarks reuse it).
    ``share_cus``: a kernel on another stream runs beside this call (a
    sharded round's all-gather): P2P_HINT_SHARE_CUS, the FedAvg split
    kernel's blocks then free CUs tile by tile (include/p2pdl.h)."""
    ref = w if w is not None else out
    if ref is None:
        raise ValueError("need w and/or out")
    N.require_device(ref)
    n = ref.numel()
    for name, t in (("w", w), ("out", out)):
        if t is not None:
            _check_f32(t, name, ref.device)
            if t.numel() != n:
                raise ValueError(f"{name} has {t.numel()} elements, expected {n}")
    r = rule_id(rule)
    k = len(peers) if table is None else table.numel()
    if table is None:
        table = _peer_inputs(peers, n, ref.device)
    else:
        table_covers(table, n)
    if r not in FEDAVG_RULES and k > MAX_ROBUST_PEERS:
        raise ValueError(f"robust rules support at most {MAX_ROBUST_PEERS} peers, got {k}")
    b = 0
    if r == P2P_RULE_TRIMMED:
        b = trim_count(k, trim_frac) if trim_b is None else int(trim_b)
    if n == 0:  # nothing to reduce (the reference's loops over empty tensors); an empty
        return  # tensor's data pointer is NULL, which the C ABI would refuse
    with torch.cuda.device(ref.device):
        N.check(N.lib().p2p_aggregate_ex_f32(table.data_ptr(), k, n, r, b, lr,
                                             w.data_ptr() if w is not None else None,
                                             out.data_ptr() if out is not None else None,
                                             N.P2P_HINT_SHARE_CUS if share_cus else 0,
                                             N.stream_handle()), "p2p_aggregate_ex_f32")


DTYPES_16 = {torch.float16: N.P2P_DTYPE_F16, torch.bfloat16: N.P2P_DTYPE_BF16}


def fedavg16_apply_(w: torch.Tensor, peers: Sequence[torch.Tensor], rule="fedavg", lr: float = 0.1) -> None:
    """FedAvg + apply in place on one float16 / bfloat16 tensor, every op
    rounded to the storage type as torch runs the reference's ops
    (aggregation.py:15-38; include/p2pdl.h p2p_fedavg_apply_16)."""
    N.require_device(w)
    dt = DTYPES_16.get(w.dtype)
    if dt is None:
        raise TypeError(f"w: expected float16 or bfloat16, got {w.dtype}")
    if not w.is_contiguous():
        raise ValueError("w: must be contiguous")
    r = rule_id(rule)
    if r not in FEDAVG_RULES:
        raise NotImplementedError(f"rule {rule!r} on a {w.dtype} model: the robust rules aggregate float32 models")
    if len(peers) == 0:
        raise ValueError("need at least one peer update")
    for i, p in enumerate(peers):
        if p.dtype != w.dtype or p.device != w.device or not p.is_contiguous() or p.numel() != w.numel():
            raise ValueError(f"peers[{i}]: expected a contiguous {w.dtype} tensor of {w.numel()} elements on "
                             f"{w.device}, got {p.dtype} {p.numel()} on {p.device}")
    if w.numel() == 0:  # nothing to do; an empty tensor's data pointer is NULL
        return
    table = pointer_table(peers, w.device)
    with torch.cuda.device(w.device):
        N.check(N.lib().p2p_fedavg_apply_16(table.data_ptr(), len(peers), w.numel(), w.data_ptr(), lr, dt, r,
                                            N.stream_handle()), "p2p_fedavg_apply_16")


def fedavg_apply_(w: torch.Tensor, peers: Sequence[torch.Tensor], lr: float = 0.1) -> torch.Tensor:
    """w += lr * mean(peers) in place (reference aggregation.py:15-38)."""
    aggregate(peers, "fedavg", w=w, lr=lr)
    return w


def mean(peers: Sequence[torch.Tensor]) -> torch.Tensor:
    out = torch.empty_like(peers[0])
    aggregate(peers, "fedavg", out=out)
    return out


def median(peers: Sequence[torch.Tensor]) -> torch.Tensor:
    out = torch.empty_like(peers[0])
    aggregate(peers, "median", out=out)
    return out


def trimmed_mean(peers: Sequence[torch.Tensor], trim_frac: float = DEFAULT_TRIM_FRAC,
                 trim_b: int | None = None) -> torch.Tensor:
    out = torch.empty_like(peers[0])
    aggregate(peers, "trimmed", out=out, trim_frac=trim_frac, trim_b=trim_b)
    return out


def apply_(w: torch.Tensor, agg: torch.Tensor, lr: float = 0.1) -> torch.Tensor:
    N.require_device(w)
    _check_f32(w, "w", w.device)
    _check_f32(agg, "agg", w.device)
    if agg.numel() != w.numel():
        raise ValueError("w and agg differ in size")
    if w.numel() == 0:
        return w
    with torch.cuda.device(w.device):
        N.check(N.lib().p2p_apply_f32(w.data_ptr(), agg.data_ptr(), lr, w.numel(),
                                      N.stream_handle()), "p2p_apply_f32")
    return w


# ----------------------------------------------------- whole state_dict
_SEG_DTYPE = np.dtype([("peers", "<u8"), ("w", "<u8"), ("out", "<u8"), ("n", "<i8"),
                       ("tile_begin", "<i8")])  # == p2p_segment_t (40 B)


class _PinnedRing:
    """Pinned host staging for the small per-call device tables (segment
    tables, pointer tables).  The table is written on the host and copied
    with a non-blocking H2D on the launch stream, so the host can build the
    next call's table while the GPU still runs this call's kernel (a pageable
    copy would wait for the stream to drain).  A slot is reused only after
    the event of the copy that last read it has completed."""

    def __init__(self, slots: int = 8):
        self.slots = [[None, None] for _ in range(slots)]  # [event, pinned uint8 buffer]
        self.i = 0
        self.lock = threading.Lock()

    def to_device(self, host: np.ndarray, dev, out: torch.Tensor | None = None) -> torch.Tensor:
        """Copy host (uint8-viewable) into `out` (a device uint8 buffer of
        host.nbytes, allocated here when None) on the current stream."""
        nbytes = host.nbytes
        with self.lock:
            slot = self.slots[self.i % len(self.slots)]
            self.i += 1
            if slot[0] is not None:
                slot[0].synchronize()
            if slot[1] is None or slot[1].numel() < nbytes:
                slot[1] = torch.empty(max(nbytes, 1 << 16), dtype=torch.uint8, pin_memory=True)
            pinned = slot[1][:nbytes]
            np.copyto(pinned.numpy(), host.view(np.uint8).reshape(-1))
            if out is None:
                out = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            with torch.cuda.device(dev):
                out.copy_(pinned, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
            slot[0] = ev
        return out


_RING = _PinnedRing()


# Device segment tables of the slab fast path, keyed by every address and
# size they encode (slab base / pitch, rows, key offsets, w pointers and
# element counts, rule, K, trim): the same inbox rows aggregated into the same
# model again -- every round of a node -- reuse the table, with no host work
# and no H2D copy.  A table holds only addresses, so an equal key means an
# equal table; entries are immutable once built.
_TABLES: "OrderedDict[tuple, tuple]" = OrderedDict()
_TABLES_MAX = 32
_TABLES_LOCK = threading.Lock()


class _NoCtx:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


_NO_CTX = _NoCtx()


def _launch_table(base: int, L: int, tiles: int, K: int, r: int, b: int, lr: float, stream=None) -> None:
    N.check(N.lib().p2p_aggregate_segments_f32(base, L, tiles, K, r, b, lr,
                                               N.stream_handle() if stream is None else stream),
            "p2p_aggregate_segments_f32")


SPLIT_TILE = 8192  # == P2P_SPLIT_TILE
# A state_dict goes to the split kernel only when its plan covers at least
# this many whole tiles (67M coordinates).  Same-box A/B (tools/seg_ab.py, K =
# 64, profiles/r05/seg): at ResNet-18's 11.7M coordinates (1280 planned tiles)
# split + segments ran 0.4-1.7% SLOWER than the VGPR segment kernel alone on
# three boxes -- the second launch over each tensor's ragged rest costs what
# the split tiles save; at 4x those shapes (5632 tiles) +0.9%, at 16x +2.5%.
SPLIT_SEGMENT_MIN_TILES = 2048
_SPLIT_DTYPE = np.dtype([("seg", "<i8"), ("c0", "<i8")])  # == p2p_split_tile_t (16 B)


def _split_plan(ptrs: np.ndarray, w_ptrs, out_ptrs, n_arr: np.ndarray, K: int, r: int):
    """FedAvg over a state_dict: which whole 8192-element tiles go to the
    LDS-DMA split kernel (include/p2pdl.h p2p_fedavg_split_segments_f32).
    Whole tiles of segments whose K peer pointers and w / out are 16-B
    aligned, taken in segment order, as many as p2p_fedavg_split_plan allows
    (whole rounds of the CU count), if that is SPLIT_SEGMENT_MIN_TILES or
    more.  Returns (taken tiles per segment, the
    split list) or None when nothing goes to the split kernel."""
    if r not in FEDAVG_RULES or K < 16:
        return None
    full = n_arr // SPLIT_TILE
    aligned = (ptrs % np.uint64(16) == 0).all(axis=1) & (np.asarray(w_ptrs, dtype=np.uint64) % np.uint64(16) == 0)
    if out_ptrs is not None:
        aligned &= np.asarray(out_ptrs, dtype=np.uint64) % np.uint64(16) == 0
    full = np.where(aligned, full, 0)
    S = int(N.lib().p2p_fedavg_split_plan(K, int(full.sum())))
    if S <= 0 or S < SPLIT_SEGMENT_MIN_TILES:
        return None
    before = np.cumsum(full) - full
    taken = np.clip(S - before, 0, full)
    seg = np.repeat(np.arange(len(n_arr), dtype=np.int64), taken)
    first = np.repeat(np.cumsum(taken) - taken, taken)
    lst = np.empty(S, dtype=_SPLIT_DTYPE)
    lst["seg"] = seg
    lst["c0"] = (np.arange(S, dtype=np.int64) - first) * SPLIT_TILE
    return taken, lst


def _chunk_plan(ptrs: np.ndarray, w_ptrs, out_ptrs, n_arr: np.ndarray, K: int, r: int):
    """FedAvg over a state_dict of separately allocated tensors on the split
    kernel in one launch (include/p2pdl.h p2p_fedavg_split_chunks_f32): every
    key whose K peer pointers and w / out are 16-B aligned, cut into
    1024-element chunks, eight chunks per split tile, the last tile padded
    (seg -1).  Taken for K >= 16 when the tiles fill at least one round of
    the CUs (p2p_fedavg_split_plan); below that the VGPR segment kernel's
    smaller blocks cover the chip better.  Returns (chunked keys mask, the
    chunk list) or None."""
    if r not in FEDAVG_RULES or K < 16:
        return None
    low = np.bitwise_or.reduce(ptrs, axis=1) | np.asarray(w_ptrs, dtype=np.uint64)
    if out_ptrs is not None:
        low |= np.asarray(out_ptrs, dtype=np.uint64)
    aligned = ((low & np.uint64(15)) == 0) & (n_arr > 0)
    nch = np.where(aligned, -(-n_arr // ROW_CHUNK), 0)
    C = int(nch.sum())
    ntiles = -(-C // (SPLIT_TILE // ROW_CHUNK))
    if ntiles == 0 or int(N.lib().p2p_fedavg_split_plan(K, ntiles)) <= 0:
        return None
    per = SPLIT_TILE // ROW_CHUNK
    M = ntiles * per
    lst = np.empty(M, dtype=_SPLIT_DTYPE)  # (seg, c0) == p2p_split_tile_t, padded with (-1, 0)
    if _host_tables.fill_chunk_list(np.ascontiguousarray(nch, dtype=np.int64), lst) != C:
        raise RuntimeError("chunk list: size mismatch")
    cus = CHUNK_BALANCE_CUS
    if cus and ntiles > cus and ntiles % cus:
        # A/B only: the chunks spread over whole CU rounds of tiles (fewer
        # chunks per tile, the rest padding) instead of a partial last round
        T = -(-ntiles // cus) * cus
        q, extra = divmod(C, T)
        cnt = np.full(T, q, dtype=np.int64)
        cnt[:extra] += 1
        slot = (np.arange(T, dtype=np.int64) * per)[:, None] + np.arange(per, dtype=np.int64)[None, :]
        take = np.arange(per)[None, :] < cnt[:, None]
        bal = np.empty(T * per, dtype=_SPLIT_DTYPE)
        bal["seg"], bal["c0"] = -1, 0
        bal[slot[take]] = lst[:C]
        lst = bal
    return aligned, lst


# A/B switch (tools/balance_ab.py): CU count to balance the chunk list over
# whole rounds of; 0 = off (the product)
CHUNK_BALANCE_CUS = 0


# How a FedAvg state_dict of separately allocated tensors runs: "chunks" (the
# product: one split launch by 1024-float chunks, _chunk_plan), "tiles"
# (round 5: whole 8192-float tiles on the split kernel, whole CU rounds,
# from SPLIT_SEGMENT_MIN_TILES up, the rest on the VGPR kernel) or "vgpr"
# (the VGPR segment kernel alone).  Same bits on every route; the others are
# kept for A/B (tools/chunks_ab.py) and their tests.
STATE_DICT_ROUTE = "chunks"


class _Layout:
    """Everything of a segment-table launch but its addresses: the plan (the
    chunk list / split tile list, which keys and ranges the VGPR kernel
    takes), the byte layout of the one device buffer and a host image with
    every address-independent field filled.  A pure function of (element
    counts, K, rule, trim, outs or not, route, the keys' 16-B alignment), so
    a round whose updates arrive at new addresses -- every round of a node
    whose listener unpickles them (node/node.py:138-141) -- reuses it and
    only writes the addresses (_LAYOUTS)."""

    __slots__ = ("tiles", "r", "b", "rem_idx", "start4", "offs", "template", "has_plan", "split", "full_rows",
                 "rem_rows", "Lr")


_LAYOUTS: "OrderedDict[tuple, _Layout]" = OrderedDict()
_LAYOUTS_MAX = 32


def _build_layout(ptrs, w_ptrs, out_ptrs, n_arr, K, r, b, tile, route):
    plan = chunks = None
    if route == "chunks":
        chunks = _chunk_plan(ptrs, w_ptrs, out_ptrs, n_arr, K, r)
    elif route == "tiles":
        plan = _split_plan(ptrs, w_ptrs, out_ptrs, n_arr, K, r)
    elif route != "vgpr":
        raise ValueError(f"unknown STATE_DICT_ROUTE {route!r}")
    L = len(n_arr)
    # The table the VGPR segment kernel runs: every segment, or -- with a
    # split plan -- what the split kernel leaves of each (its tail past the
    # taken whole tiles), as segments of their own whose peer rows, w and out
    # start at that offset; with a chunk plan, the keys it could not take.
    if chunks is not None:
        rem_idx = np.nonzero(~chunks[0] & (n_arr > 0))[0]
        start = np.zeros(len(rem_idx), dtype=np.int64)
        plan = (None, chunks[1])
    elif plan is None:
        rem_idx, start = np.arange(L), np.zeros(L, dtype=np.int64)
    else:
        taken = plan[0]
        start = taken * SPLIT_TILE
        rem_idx = np.nonzero(n_arr - start > 0)[0]
        start = start[rem_idx]
    lay = _Layout()
    lay.r, lay.b = r, b
    lay.Lr = Lr = len(rem_idx)
    lay.rem_idx, lay.start4 = rem_idx, start.astype(np.uint64) * np.uint64(4)
    rem = np.zeros(Lr, dtype=_SEG_DTYPE)
    rem["n"] = n_arr[rem_idx] - start
    t_arr = -(-rem["n"] // tile)
    if Lr:
        rem["tile_begin"][1:] = np.cumsum(t_arr)[:-1]
    lay.tiles = int(t_arr.sum())
    lay.has_plan = plan is not None
    if lay.tiles == 0 and plan is None:
        lay.template = None  # nothing to launch
        return lay
    # one device buffer: [the full table (split kernel's segments)] [the
    # remainder table] [split tile list] [full peer rows] [remainder peer
    # rows].  Its tables hold device addresses inside itself: the launch
    # allocates it first, then writes those addresses into a copy of the
    # template and copies it once.
    full = np.zeros(L if plan is not None else 0, dtype=_SEG_DTYPE)
    lst = plan[1] if plan is not None else np.zeros(0, dtype=_SPLIT_DTYPE)
    parts = [full.nbytes, rem.nbytes, lst.nbytes, 8 * K * len(full), 8 * K * Lr]
    offs = np.concatenate([[0], np.cumsum(parts)]).astype(np.int64)
    lay.offs = [int(x) for x in offs]
    host = np.zeros(lay.offs[-1], dtype=np.uint8)
    if plan is not None:
        full["n"] = n_arr
        host[offs[0]:offs[1]] = full.view(np.uint8)
        host[offs[2]:offs[3]] = lst.view(np.uint8)
    host[offs[1]:offs[2]] = rem.view(np.uint8)
    lay.template = host
    lay.full_rows = np.uint64(offs[3]) + np.arange(len(full), dtype=np.uint64) * np.uint64(8 * K)
    lay.rem_rows = np.uint64(offs[4]) + np.arange(Lr, dtype=np.uint64) * np.uint64(8 * K)
    if plan is None:
        lay.split = None
    elif chunks is not None:  # the chunk list: ntiles * 8 entries
        lay.split = (lay.offs[2], len(lst) // (SPLIT_TILE // ROW_CHUNK), lay.offs[0], "chunks")
    else:
        lay.split = (lay.offs[2], len(lst), lay.offs[0], "tiles")
    return lay


def _launch_segments(ws, ptrs: np.ndarray, numels, rule, K, lr, trim_b, trim_frac, outs, dev, cache_key=None):
    r = rule_id(rule)
    if r not in FEDAVG_RULES and K > MAX_ROBUST_PEERS:
        raise ValueError(f"robust rules support at most {MAX_ROBUST_PEERS} peers, got {K}")
    b = trim_count(K, trim_frac) if (r == P2P_RULE_TRIMMED and trim_b is None) else int(trim_b or 0)
    n_arr = np.asarray(numels, dtype=np.int64)
    w_arr = np.fromiter((w.data_ptr() for w in ws), dtype=np.uint64, count=len(ws))
    out_arr = np.fromiter((o.data_ptr() for o in outs), dtype=np.uint64, count=len(outs)) if outs is not None else None
    ptrs = np.ascontiguousarray(ptrs, dtype=np.uint64)
    route = STATE_DICT_ROUTE
    mask = None  # the keys' 16-B alignment, where a split plan depends on it
    if route != "vgpr" and r in FEDAVG_RULES and K >= 16 and len(n_arr):
        low = np.bitwise_or.reduce(ptrs, axis=1) | w_arr
        if out_arr is not None:
            low |= out_arr
        mask = ((low & np.uint64(15)) == 0).tobytes()
    lkey = (dev.index, n_arr.tobytes(), K, r, b, out_arr is not None, route, mask)
    with _TABLES_LOCK:
        lay = _LAYOUTS.get(lkey)
        if lay is not None:
            _LAYOUTS.move_to_end(lkey)
    if lay is None:
        lay = _build_layout(ptrs, w_arr, out_arr, n_arr, K, r, b, int(N.lib().p2p_tile_elems(r, K)), route)
        with _TABLES_LOCK:
            _LAYOUTS[lkey] = lay
            while len(_LAYOUTS) > _LAYOUTS_MAX:
                _LAYOUTS.popitem(last=False)
    if lay.template is None:
        return None
    o = lay.offs
    host = lay.template.copy()
    buf = torch.empty(host.nbytes, dtype=torch.uint8, device=dev)
    base = np.uint64(buf.data_ptr())
    if lay.has_plan:
        full = host[o[0]:o[1]].view(_SEG_DTYPE)
        full["w"] = w_arr
        if out_arr is not None:
            full["out"] = out_arr
        full["peers"] = base + lay.full_rows
        host[o[3]:o[4]] = ptrs.view(np.uint8).reshape(-1)
    if lay.Lr:
        rem = host[o[1]:o[2]].view(_SEG_DTYPE)
        ri = lay.rem_idx
        rem["w"] = w_arr[ri] + lay.start4
        if out_arr is not None:
            rem["out"] = out_arr[ri] + lay.start4
        rem["peers"] = base + lay.rem_rows
        host[o[4]:o[5]] = (ptrs[ri] + lay.start4[:, None]).view(np.uint8).reshape(-1)
    _RING.to_device(host, dev, out=buf)
    entry = (buf, lay.tiles, r, b, torch.cuda.current_stream(dev).cuda_stream, (o[1], lay.Lr, lay.split))
    with torch.cuda.device(dev):
        _launch_entry(entry, K, lr, N.stream_handle())
    if cache_key is not None:
        with _TABLES_LOCK:
            _TABLES[cache_key] = entry
            while len(_TABLES) > _TABLES_MAX:
                _TABLES.popitem(last=False)
        return entry
    return None


ROW_CHUNK = 1024  # == P2P_ROW_CHUNK
_CHUNK_DTYPE = np.dtype([("w", "<u8"), ("valid", "<i8")])  # == p2p_row_chunk_t (16 B)


def _rows_entry(ws, w_ptrs, numels, slab, rows_a, offs_a, r, K, lr, dev, cache_key):
    """FedAvg over slab rows as flat peers (include/p2pdl.h
    p2p_fedavg_split_rows_f32): one split launch over whole tiles of the rows,
    the model scattered by 1024-float chunks.  Taken when every key starts a
    1024-float boundary (DeviceInbox's chunk layout), the rows hold whole
    tiles, the w tensors are 16-B aligned and the tiles fill at least one
    round of the CUs (the split plan); otherwise None (the segment path)."""
    if r not in FEDAVG_RULES:
        return None
    n_a = np.asarray(numels, dtype=np.int64)
    if (offs_a % ROW_CHUNK).any() or (np.asarray(w_ptrs, dtype=np.uint64) % np.uint64(16)).any():
        return None
    width = slab.shape[1]
    ntiles = -(-int((offs_a + n_a).max()) // SPLIT_TILE)
    if ntiles * SPLIT_TILE > width or (width * 4) % 16 or slab.data_ptr() % 16:
        return None
    if int(N.lib().p2p_fedavg_split_plan(K, ntiles)) <= 0:  # below one round (or K < 16)
        return None
    order = np.argsort(offs_a, kind="stable")
    ends = offs_a[order] + n_a[order]
    if (offs_a[order][1:] < ends[:-1]).any():  # overlapping keys: no chunk map
        return None
    chunks = np.zeros(ntiles * (SPLIT_TILE // ROW_CHUNK), dtype=_CHUNK_DTYPE)
    for l in range(len(ws)):
        n = int(n_a[l])
        if n == 0:
            continue
        c0, c1 = int(offs_a[l]) // ROW_CHUNK, -(-(int(offs_a[l]) + n) // ROW_CHUNK)
        j = np.arange(c1 - c0, dtype=np.int64)
        chunks["w"][c0:c1] = np.uint64(w_ptrs[l]) + (j * ROW_CHUNK * 4).astype(np.uint64)
        chunks["valid"][c0:c1] = np.minimum(ROW_CHUNK, n - j * ROW_CHUNK)
    row_ptrs = np.uint64(slab.data_ptr()) + rows_a.astype(np.uint64) * np.uint64(width * 4)
    host = np.concatenate([row_ptrs.view(np.uint8), chunks.view(np.uint8)])
    buf = torch.empty(host.nbytes, dtype=torch.uint8, device=dev)
    _RING.to_device(host, dev, out=buf)
    entry = (buf, 0, r, 0, torch.cuda.current_stream(dev).cuda_stream, ("rows", row_ptrs.nbytes, ntiles))
    with torch.cuda.device(dev):
        _launch_entry(entry, K, lr, N.stream_handle())
    with _TABLES_LOCK:
        _TABLES[cache_key] = entry
        while len(_TABLES) > _TABLES_MAX:
            _TABLES.popitem(last=False)
    return entry


def _launch_entry(entry, K: int, lr: float, stream) -> None:
    """The launches of one segment-table entry: the rows kernel (a slab's rows
    as flat peers), or the split kernel over its tile list (when planned),
    then the VGPR segment kernel over the rest."""
    buf, tiles, r, b, _, extra = entry
    base = buf.data_ptr()
    if extra[0] == "rows":
        _, ch_off, ntiles = extra
        N.check(N.lib().p2p_fedavg_split_rows_f32(base, K, ntiles, base + ch_off, r, lr, stream),
                "p2p_fedavg_split_rows_f32")
        return
    rem_off, Lr, split = extra
    if split is not None:
        lst_off, S, segs_off, how = split
        if how == "chunks":
            N.check(N.lib().p2p_fedavg_split_chunks_f32(base + lst_off, S, base + segs_off, K, r, lr, stream),
                    "p2p_fedavg_split_chunks_f32")
        else:
            N.check(N.lib().p2p_fedavg_split_segments_f32(base + lst_off, S, base + segs_off, K, r, lr, stream),
                    "p2p_fedavg_split_segments_f32")
    if tiles:
        _launch_table(base + rem_off, Lr, tiles, K, r, b, lr, stream=stream)


def aggregate_segments_(ws: Sequence[torch.Tensor], peer_lists: Sequence[Sequence[torch.Tensor]],
                        rule="fedavg", *, lr: float = 0.1, trim_b: int | None = None,
                        trim_frac: float = DEFAULT_TRIM_FRAC,
                        outs: Sequence[torch.Tensor] | None = None) -> None:
    """All L tensors of a state_dict in ONE launch.

    ws[l] is updated in place with lr * rule(peer_lists[j][l] for j in peers);
    peer_lists[j] is the j-th update's tensors in the same key order."""
    L = len(ws)
    if L == 0:
        return
    K = len(peer_lists)
    if K == 0:
        raise ValueError("need at least one peer update")
    dev = ws[0].device
    N.require_device(ws[0])
    for l, w in enumerate(ws):
        _check_f32(w, f"w[{l}]", dev)
    if outs is not None:
        for l, (o, w) in enumerate(zip(outs, ws)):
            _check_f32(o, f"out[{l}]", dev)
            if o.numel() != w.numel():
                raise ValueError(f"out[{l}] has {o.numel()} elements, expected {w.numel()}")
    numels = [w.numel() for w in ws]
    di = dev.index
    f32 = torch.float32
    ptrs = np.empty((L, K), dtype=np.uint64)
    for j, row in enumerate(peer_lists):
        if len(row) != L:
            raise ValueError(f"update[{j}] has {len(row)} tensors, expected {L}")
        # one pass of cheap C getters per tensor; the detailed error (same
        # checks as _check_f32) only when something is off
        if not all(t.dtype is f32 and t.get_device() == di and t.is_contiguous() and t.numel() == n
                   for t, n in zip(row, numels)):
            for l, (t, n) in enumerate(zip(row, numels)):
                _check_f32(t, f"update[{j}][{l}]", dev)
                if t.numel() != n:
                    raise ValueError(f"update[{j}][{l}] has {t.numel()} elements, expected {n}")
        ptrs[:, j] = [t.data_ptr() for t in row]
    _launch_segments(ws, ptrs, numels, rule, K, lr, trim_b, trim_frac, outs, dev)


def aggregate_ptr_table_(ws: Sequence[torch.Tensor], ptrs: np.ndarray, rule="fedavg", *, lr: float = 0.1,
                         trim_b: int | None = None, trim_frac: float = DEFAULT_TRIM_FRAC,
                         w_ptrs: tuple | None = None, numels: tuple | None = None) -> None:
    """aggregate_segments_ for a peer-pointer table the caller has already
    gathered and validated: ptrs[l, j] = device address of update j's
    fp32 tensor for key l (ws[l].numel() elements each, contiguous, on ws'
    device) -- what _host_tables.gather_peer_table returns for
    aggregate_models' general path.  The device table is cached by the
    addresses and sizes it encodes (a round whose updates land at the same
    addresses reuses it, as aggregate_slab_rows_ does).  ``w_ptrs`` /
    ``numels``: caller-validated, as for aggregate_slab_rows_."""
    L = len(ws)
    if L == 0:
        return
    if ptrs.shape[0] != L or ptrs.shape[1] == 0 or ptrs.dtype != np.uint64:
        raise ValueError("ptrs must be a uint64 [L, K] table, K >= 1")
    K = ptrs.shape[1]
    dev = ws[0].device
    N.require_device(ws[0])
    if w_ptrs is None:
        for l, w in enumerate(ws):
            _check_f32(w, f"w[{l}]", dev)
        w_ptrs = tuple(w.data_ptr() for w in ws)
    if numels is None:
        numels = tuple(w.numel() for w in ws)
    key = (dev.index, "ptrs", ptrs.tobytes(), w_ptrs, numels, rule_id(rule), K, trim_b, float(trim_frac))
    with _TABLES_LOCK:
        hit = _TABLES.get(key)
        if hit is not None:
            _TABLES.move_to_end(key)
    if hit is not None:
        _relaunch(hit, dev, K, lr)
        return
    _launch_segments(ws, ptrs, numels, rule, K, lr, trim_b, trim_frac, None, dev, cache_key=key)


def aggregate_slab_rows_(ws: Sequence[torch.Tensor], slab: torch.Tensor, rows: Sequence[int],
                         offsets: Sequence[int], rule="fedavg", *, lr: float = 0.1,
                         trim_b: int | None = None, trim_frac: float = DEFAULT_TRIM_FRAC,
                         w_ptrs: tuple | None = None, numels: tuple | None = None):
    """aggregate_segments_ for updates that are rows of one [K_max, N] fp32
    slab (what node.inbox.DeviceInbox lands): update j's tensor for key l is
    slab[rows[j], offsets[l] : offsets[l] + ws[l].numel()].  The (L, K) peer
    table is computed with one broadcast instead of inspecting L*K tensors.
    ``w_ptrs``: the ws' data pointers, from a caller that has already checked
    ws (fp32, contiguous, on the slab's device) and vouches they are
    unchanged (aggregation.py's validated model-state cache); the per-tensor
    checks are then skipped (``numels``: their element counts, likewise).
    Returns the device-table cache entry it launched (``relaunch`` takes
    it), or None when there was nothing to launch."""
    L, K = len(ws), len(rows)
    if L == 0:
        return
    if K == 0:
        raise ValueError("need at least one peer update")
    dev = slab.device
    N.require_device(slab)
    if slab.dtype != torch.float32 or slab.dim() != 2 or not slab.is_contiguous():
        raise ValueError("slab must be a contiguous fp32 [K_max, N] tensor")
    if w_ptrs is None:
        for l, w in enumerate(ws):
            _check_f32(w, f"w[{l}]", dev)
        w_ptrs = tuple(w.data_ptr() for w in ws)
    if numels is None:
        numels = tuple(w.numel() for w in ws)
    key = (dev.index, slab.data_ptr(), slab.shape[0], slab.shape[1], tuple(rows), tuple(offsets),
           w_ptrs, numels, rule_id(rule), K, trim_b, float(trim_frac))
    with _TABLES_LOCK:
        hit = _TABLES.get(key)
        if hit is not None:
            _TABLES.move_to_end(key)
    if hit is not None:  # same addresses and sizes as a previous call: same table
        relaunch(hit, dev, L, K, lr)
        return hit
    rows_a = np.asarray(rows, dtype=np.int64)
    offs_a = np.asarray(offsets, dtype=np.int64)
    kmax, width = slab.shape
    if rows_a.min() < 0 or rows_a.max() >= kmax:
        raise IndexError("slab row out of range")
    if offs_a.min() < 0 or (offs_a + np.asarray(numels, dtype=np.int64)).max() > width:
        raise IndexError("segment outside the slab row")
    entry = _rows_entry(ws, w_ptrs, numels, slab, rows_a, offs_a, rule_id(rule), K, lr, dev, key)
    if entry is not None:
        return entry
    base, stride = slab.data_ptr(), width * 4
    ptrs = (np.uint64(base) + rows_a.astype(np.uint64)[None, :] * np.uint64(stride)
            + offs_a.astype(np.uint64)[:, None] * np.uint64(4))
    return _launch_segments(ws, ptrs, numels, rule, K, lr, trim_b, trim_frac, None, dev, cache_key=key)


def relaunch(entry, dev, L: int, K: int, lr: float) -> None:
    """Launch a cached device segment table again (an entry that
    aggregate_slab_rows_ / aggregate_ptr_table_ returned): the same kernel
    over the same addresses, on the current stream of ``dev`` -- no table
    work, no H2D copy, no per-call checks (the caller vouches that the
    addresses it was built from are unchanged)."""
    _relaunch(entry, dev, K, lr)


def _relaunch(entry, dev, K: int, lr: float) -> None:
    buf, alloc_stream = entry[0], entry[4]
    with torch.cuda.device(dev) if torch.cuda.current_device() != dev.index else _NO_CTX:
        raw = N.stream_handle(dev.index)
        if raw != alloc_stream:
            buf.record_stream(torch.cuda.current_stream(dev))  # eviction must not recycle it under this launch
        _launch_entry(entry, K, lr, raw)


# ------------------------------------------------------------------ K4
DELTA_TILE = 1024  # == P2P_DELTA_TILE
_DSEG_DTYPE = np.dtype([("cur", "<u8"), ("prev", "<u8"), ("delta", "<u8"), ("n", "<i8"),
                        ("tile_begin", "<i8")])  # == p2p_delta_segment_t (40 B)


def delta_snapshot_(cur: torch.Tensor, prev: torch.Tensor, delta: torch.Tensor, first: bool = False) -> None:
    """delta = cur - prev; prev = cur (first: delta = cur), one pass
    (reference node/node.py:273-282 for one flat buffer)."""
    N.require_device(cur)
    for name, t in (("cur", cur), ("prev", prev), ("delta", delta)):
        _check_f32(t, name, cur.device)
        if t.numel() != cur.numel():
            raise ValueError(f"{name} has {t.numel()} elements, expected {cur.numel()}")
    if cur.numel() == 0:
        return
    with torch.cuda.device(cur.device):
        N.check(N.lib().p2p_delta_snapshot_f32(cur.data_ptr(), prev.data_ptr(), delta.data_ptr(), cur.numel(),
                                               int(first), N.stream_handle()), "p2p_delta_snapshot_f32")


def delta_snapshot_segments_(curs: Sequence[torch.Tensor], prevs: Sequence[torch.Tensor],
                             deltas: Sequence[torch.Tensor], first: bool = False) -> None:
    """Whole state_dict in ONE launch: deltas[l] = curs[l] - prevs[l]; prevs[l] = curs[l]."""
    L = len(curs)
    if L == 0:
        return
    if not (len(prevs) == len(deltas) == L):
        raise ValueError("curs, prevs and deltas must have the same length")
    dev = curs[0].device
    N.require_device(curs[0])
    segs = np.zeros(L, dtype=_DSEG_DTYPE)
    tiles = 0
    for l, (c, p, d) in enumerate(zip(curs, prevs, deltas)):
        for name, t in (("cur", c), ("prev", p), ("delta", d)):
            _check_f32(t, f"{name}[{l}]", dev)
            if t.numel() != c.numel():
                raise ValueError(f"{name}[{l}] has {t.numel()} elements, expected {c.numel()}")
        segs[l] = (c.data_ptr(), p.data_ptr(), d.data_ptr(), c.numel(), tiles)
        tiles += -(-c.numel() // DELTA_TILE)
    if tiles == 0:
        return
    buf = _RING.to_device(segs.view(np.uint8), dev)
    with torch.cuda.device(dev):
        N.check(N.lib().p2p_delta_snapshot_segments_f32(buf.data_ptr(), L, tiles, int(first), N.stream_handle()),
                "p2p_delta_snapshot_segments_f32")
    buf.record_stream(torch.cuda.current_stream(dev))


# ------------------------------------------------------------------ K3
def _check_tensor(t: torch.Tensor, name: str, dtypes, shape, dev, min_numel: int = 0) -> None:
    dtypes = dtypes if isinstance(dtypes, tuple) else (dtypes,)
    if t.dtype not in dtypes or not t.is_contiguous() or t.device != dev:
        raise ValueError(f"{name} must be a contiguous {'/'.join(str(d) for d in dtypes)} tensor on {dev}, "
                         f"got {t.dtype} on {t.device}")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} has shape {tuple(t.shape)}, expected {tuple(shape)}")
    if t.numel() < min_numel:
        raise ValueError(f"{name} has {t.numel()} elements, needs at least {min_numel}")


def check_message_spans(msgs: torch.Tensor, offsets: Sequence[int], lengths: Sequence[int]) -> None:
    """Messages [offset, offset + length) of a contiguous 1-D uint8 buffer:
    raises ValueError for any span outside it."""
    if msgs.dtype != torch.uint8 or msgs.dim() != 1 or not msgs.is_contiguous():
        raise ValueError(f"messages must be a contiguous 1-D uint8 tensor, got {msgs.dtype} {tuple(msgs.shape)}")
    if len(offsets) != len(lengths):
        raise ValueError(f"{len(offsets)} offsets for {len(lengths)} lengths")
    size = msgs.numel()
    for j, (o, n) in enumerate(zip(offsets, lengths)):
        o, n = int(o), int(n)
        if o < 0 or n < 0 or o + n > size:
            raise ValueError(f"message {j}: bytes [{o}, {o + n}) outside the {size}-byte buffer")


def sha256_batch_device(msgs: torch.Tensor, offsets: Sequence[int], lengths: Sequence[int]) -> torch.Tensor:
    """Digest K messages that live in one device uint8 buffer.

    Returns a (K, 32) uint8 device tensor; does not synchronise.  Every
    message must lie inside ``msgs`` (ValueError otherwise: the kernel reads
    raw addresses)."""
    N.require_device(msgs)
    check_message_spans(msgs, offsets, lengths)
    dev = msgs.device
    K = len(offsets)
    digests = torch.empty((max(K, 1), 32), dtype=torch.uint8, device=dev)
    if K == 0:
        return digests[:0]
    base = msgs.data_ptr()
    tab = _RING.to_device(np.array([[base + int(o) for o in offsets], [int(x) for x in lengths]],
                                   dtype=np.int64), dev).view(torch.int64)
    ptrs, lens = tab[:K], tab[K:]
    with torch.cuda.device(dev):
        N.check(N.lib().p2p_sha256_batch(ptrs.data_ptr(), lens.data_ptr(), K, digests.data_ptr(),
                                         N.stream_handle()), "p2p_sha256_batch")
    return digests


def pack_messages(messages: Iterable[bytes], align: int = 16):
    """Concatenate byte strings at `align`-byte offsets into one host buffer."""
    messages = list(messages)
    offsets, o = [], 0
    for m in messages:
        offsets.append(o)
        o += -(-max(len(m), 1) // align) * align
    host = np.zeros(max(o, align), dtype=np.uint8)
    for off, m in zip(offsets, messages):
        if m:
            host[off:off + len(m)] = np.frombuffer(m, dtype=np.uint8)
    return host, offsets, [len(m) for m in messages]


def sha256_batch(messages: Sequence[bytes], device=None) -> list[bytes]:
    """SHA-256 of every message on the GPU (one H2D copy, one launch)."""
    if device is None:
        if not torch.cuda.is_available():
            raise N.NativeUnavailable("p2pdl_amd: no ROCm GPU visible; the HIP hot path cannot run")
        device = torch.device("cuda", torch.cuda.current_device())
    host, offsets, lens = pack_messages(messages)
    dev_buf = torch.from_numpy(host).to(device)
    d = sha256_batch_device(dev_buf, offsets, lens).cpu().numpy()
    return [bytes(d[i]) for i in range(len(lens))]


def digest_accept(digests: torch.Tensor, expected: torch.Tensor, payload_table: torch.Tensor,
                  accepted: torch.Tensor, count: torch.Tensor) -> None:
    """accepted[0:count] = payloads whose digest matches, in list order (device).
    Shapes are checked here (the kernel reads raw addresses): digests and
    expected (k, 32) uint8, payload_table / accepted k 8-byte pointers,
    count one int32, all on one device."""
    k = payload_table.numel()
    dev = digests.device
    _check_tensor(digests, "digests", torch.uint8, (k, 32), dev)
    _check_tensor(expected, "expected", torch.uint8, (k, 32), dev)
    _check_tensor(payload_table, "payload_table", (torch.int64, torch.uint64), (k,), dev)
    _check_tensor(accepted, "accepted", (torch.int64, torch.uint64), None, dev, min_numel=k)
    _check_tensor(count, "count", torch.int32, None, dev, min_numel=1)
    with torch.cuda.device(digests.device):
        N.check(N.lib().p2p_digest_accept(digests.data_ptr(), expected.data_ptr(),
                                          payload_table.data_ptr(), k, accepted.data_ptr(),
                                          count.data_ptr(), N.stream_handle()), "p2p_digest_accept")


def fedavg_apply_devk_(w: torch.Tensor, table: torch.Tensor, k_dev: torch.Tensor, k_max: int,
                       lr: float = 0.1, out: torch.Tensor | None = None) -> None:
    """FedAvg over table[0:*k_dev] with the peer count read on the device
    (1 <= *k_dev <= k_max, the caller's contract: the count is not read on
    the host).  table holds at least k_max 8-byte pointers."""
    dev = w.device
    _check_f32(w, "w", dev)
    if out is not None:
        _check_f32(out, "out", dev)
        if out.numel() != w.numel():
            raise ValueError(f"out has {out.numel()} elements, w {w.numel()}")
    if not 1 <= k_max:
        raise ValueError(f"k_max must be >= 1, got {k_max}")
    _check_tensor(table, "table", (torch.int64, torch.uint64), None, dev, min_numel=k_max)
    table_covers(table, w.numel())
    _check_tensor(k_dev, "k_dev", torch.int32, None, dev, min_numel=1)
    if w.numel() == 0:
        return
    with torch.cuda.device(w.device):
        N.check(N.lib().p2p_fedavg_apply_devk_f32(table.data_ptr(), k_dev.data_ptr(), k_max, w.numel(),
                                                  w.data_ptr(), lr,
                                                  out.data_ptr() if out is not None else None,
                                                  N.stream_handle()), "p2p_fedavg_apply_devk_f32")


# ------------------------------------------------------------- synthetic
def fill_synthetic_(out: torch.Tensor, seed: int, peer: int, scale: float, chunk: int = 0,
                    nranks: int = 1, rank: int = 0) -> torch.Tensor:
    N.require_device(out)
    _check_f32(out, "out", out.device)
    if out.numel() == 0:
        return out
    with torch.cuda.device(out.device):
        N.check(N.lib().p2p_fill_synthetic_f32(out.data_ptr(), out.numel(), seed, peer, scale,
                                               chunk, nranks, rank, N.stream_handle()),
                "p2p_fill_synthetic_f32")
    return out
