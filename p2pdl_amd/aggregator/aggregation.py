"""Drop-in for reference ``aggregator/aggregation.py``.

``aggregate_models(self)`` keeps the reference's name, signature and
behaviour (reference aggregator/aggregation.py:7-46); node/node.py:12 can
import it (and ``broadcast_global_model_update``) from here unchanged and call
it from ``Node.testing`` (node/node.py:316).  The per-key torch op loops of the
reference are replaced by ONE launch of the gfx950 segment kernel over the
whole state_dict (include/p2pdl.h ``p2p_aggregate_segments_f32``).

Semantics preserved:
  * wait for len(trainers_list) updates first (:9-10);
  * K = len(received_models) (:18); K == 0 logs an error and returns None
    without clearing or broadcasting (:20-22);
  * keys come from self.model.state_dict() (:15,:27): an update missing one
    raises KeyError, extra keys are ignored;
  * a non-floating tensor in the state_dict raises the reference's
    RuntimeError (it fails at the true division, :32) before anything changes;
  * sum in received_models list order from +0, IEEE division by K,
    w += fp32(0.1) * mean with the multiply and add separately rounded
    (:25-38) -- bit-exact with the reference on CPU;
  * then received_models.clear() (:43) and broadcast (:46).
Build extensions (keyword-only, defaults reproduce the reference): ``rule``
('fedavg' | 'median' | 'trimmed', README.md:10 "Byzantine fault" TODO, or
'fedavg_torch_gpu': FedAvg bit-exact with the reference as torch runs it on
GPU tensors -- its deployment, node/node.py:28-29 -- where :32 is
acc * fl(1/K)), ``lr`` (:36) and ``trim_frac``.
"""
import contextlib
import logging
import pickle
import socket
import weakref

import numpy as np
import torch

from .. import ops
from .._native import host_extension
from ..node import envelope
from ..node.inbox import LandedUpdate
from ..utils.waiting import wait_for_models
from .model_state import model_state

# host-side C gather of the peer table (p2pdl_amd/csrc/host_tables.cpp); no
# silent fallback when it is not built (NativeUnavailable at import)
_host_tables = host_extension("_host_tables")

LEARNING_RATE = 0.1       # reference aggregation.py:36
AGGREGATION_RULE = "fedavg"
TRIM_FRAC = 0.2

_TORCH_TYPE_NAMES = {torch.int64: "Long", torch.int32: "Int", torch.int16: "Short",
                     torch.int8: "Char", torch.uint8: "Byte", torch.bool: "Bool"}


def aggregate_models(self, *, rule=None, lr=LEARNING_RATE, trim_frac=TRIM_FRAC):
    if not wait_for_models(self.received_models, len(self.trainers_list)):
        logging.warning(f"[{self.addr}:{self.port}] Proceeding with aggregation despite incomplete models.")

    logging.debug(f"[{self.addr}:{self.port}] Aggregating local model updates ...")

    # Listener threads may still append (node/node.py:141): aggregate a snapshot.
    received = list(self.received_models)
    num_updates = len(received)
    if num_updates == 0:
        logging.error(f"[{self.addr}:{self.port}] No updates received to aggregate!")
        return

    # keys and tensors of self.model.state_dict() (:15,:27,:37), from a cache
    # re-validated against the model on every call (model_state.py)
    keys, ws, st = model_state(self.model)
    if ws and ws[0].dtype in ops.DTYPES_16:  # a float16 / bfloat16 model (e.g. model.half())
        _aggregate_16(keys, ws, received, rule or AGGREGATION_RULE, lr)
        logging.info(f"[{self.addr}:{self.port}] Model aggregation completed, applied local updates.")
        self.received_models.clear()
        broadcast_global_model_update(self)
        return
    if _slab_fast_path(st, keys, ws, received, rule or AGGREGATION_RULE, lr, trim_frac):
        logging.info(f"[{self.addr}:{self.port}] Model aggregation completed, applied local updates.")
        self.received_models.clear()
        broadcast_global_model_update(self)
        return
    # The (L, K) peer table gathered in C when every update tensor is a plain
    # fp32 tensor on the model's device (KeyError on a missing key, like :28);
    # otherwise the per-tensor path below, with the exact diagnosis.
    table = _gather_table(received, keys, ws)
    if table is None:
        updates = []
        for received_model in received:  # KeyError on a missing key, like :28
            local_update = received_model["model"]
            updates.append([local_update[key] for key in keys])

    contiguous = _check_model(keys, ws, st)

    if table is not None:
        if contiguous:  # the validated model-state entry vouches for the pointers
            with _consuming(received):
                ops.aggregate_ptr_table_(ws, table, rule or AGGREGATION_RULE, lr=lr, trim_frac=trim_frac,
                                         w_ptrs=st.ptrs if st is not None else None,
                                         numels=st.numels if st is not None else None)
            logging.info(f"[{self.addr}:{self.port}] Model aggregation completed, applied local updates.")
            self.received_models.clear()
            broadcast_global_model_update(self)
            return
        ws_c = [w if w.is_contiguous() else w.contiguous() for w in ws]
        with _consuming(received):
            ops.aggregate_ptr_table_(ws_c, table, rule or AGGREGATION_RULE, lr=lr, trim_frac=trim_frac)
        for w, wc in zip(ws, ws_c):
            if wc is not w:
                w.copy_(wc)
        logging.info(f"[{self.addr}:{self.port}] Model aggregation completed, applied local updates.")
        self.received_models.clear()
        broadcast_global_model_update(self)
        return
    numels = [w.numel() for w in ws]
    dev = ws[0].device if ws else None
    di = dev.index if dev is not None else None
    f32 = torch.float32
    peer_lists = []
    for j, row in enumerate(updates):
        # one pass of cheap getters; the per-tensor diagnosis and the exact
        # widening of fp16 / bf16 / integer updates only when needed
        if not all(u.dtype is f32 and u.get_device() == di and u.numel() == n and u.is_contiguous()
                   for u, n in zip(row, numels)):
            row = [_checked_update(j, key, w, u) for key, w, u in zip(keys, ws, row)]
        peer_lists.append(row)

    # state_dict() tensors are views of the parameters: updating them in place
    # updates the model, exactly like the reference's `+=` at :38.
    ws_c = [w if w.is_contiguous() else w.contiguous() for w in ws]
    with _consuming(received):
        ops.aggregate_segments_(ws_c, peer_lists, rule or AGGREGATION_RULE, lr=lr, trim_frac=trim_frac)
    for w, wc in zip(ws, ws_c):
        if wc is not w:
            w.copy_(wc)

    logging.info(f"[{self.addr}:{self.port}] Model aggregation completed, applied local updates.")

    # Clear received models for the next round (:43)
    self.received_models.clear()

    # Broadcast the newly aggregated global model (:46)
    broadcast_global_model_update(self)


def _aggregate_16(keys, ws, received, rule, lr) -> None:
    """A float16 / bfloat16 model: every op of :15-38 in fp32, rounded to the
    storage type, as torch runs them (ops.fedavg16_apply_, one launch per
    tensor).  Everything is checked before the first launch: a missing key
    raises KeyError (:28), an integer tensor the reference's RuntimeError
    (:32); a model mixing dtypes, updates of another dtype or a robust rule
    raise NotImplementedError."""
    _check_integers(keys, ws)
    dt = ws[0].dtype
    for key, t in zip(keys, ws):
        if t.dtype != dt:
            raise NotImplementedError(f"p2pdl_amd aggregates float32 models or uniform float16 / bfloat16 ones; "
                                      f"{key} is {t.dtype}, {keys[0]} {dt}")
    if ops.rule_id(rule) not in ops.FEDAVG_RULES:
        raise NotImplementedError(f"rule {rule!r} on a {dt} model: the robust rules aggregate float32 models")
    updates = [[received_model["model"][key] for key in keys] for received_model in received]  # KeyError (:28)
    columns = []
    for key, w, col in zip(keys, ws, zip(*updates)):
        peers = []
        for j, u in enumerate(col):
            if u.dtype != dt:
                raise NotImplementedError(f"update {j}, {key}: {u.dtype} into a {dt} model")
            if u.device != w.device:
                raise RuntimeError(f"Expected all tensors to be on the same device, but found at least two "
                                   f"devices, {w.device} and {u.device}!")
            if u.shape != w.shape:
                raise RuntimeError(f"update {j}, {key}: shape {tuple(u.shape)} != {tuple(w.shape)}")
            peers.append(u if u.is_contiguous() else u.contiguous())
        columns.append(peers)
    for w, peers in zip(ws, columns):
        wc = w if w.is_contiguous() else w.contiguous()
        with _consuming(received):
            ops.fedavg16_apply_(wc, peers, rule, lr)
        if wc is not w:
            w.copy_(wc)


def _check_integers(keys, ws) -> None:
    """The reference raises at the division for integer tensors (:32)."""
    for t in ws:
        if not t.is_floating_point():
            name = _TORCH_TYPE_NAMES.get(t.dtype, str(t.dtype))
            raise RuntimeError(f"result type Float can't be cast to the desired output type {name}")


def _check_model(keys, ws, st) -> bool:
    """The reference raises at the division for integer tensors (:32);
    a float32 model (16-bit ones take _aggregate_16; float64 and mixed
    models are not aggregated here).  Returns whether every
    model tensor is contiguous.  Decided once per validated model-state
    entry (its tensors cannot change dtype or layout while it is valid)."""
    done = st.extra.get("checked") if st is not None else None
    if done is not None:
        return done
    _check_integers(keys, ws)
    for key, t in zip(keys, ws):
        if t.dtype != torch.float32:
            raise NotImplementedError(f"p2pdl_amd aggregates float32 models or uniform float16 / bfloat16 "
                                      f"ones; {key} is {t.dtype}")
    contiguous = all(t.is_contiguous() for t in ws)
    if st is not None:
        st.extra["checked"] = contiguous
    return contiguous


def _gather_table(received, keys, ws):
    """uint64 [L, K] device addresses of received[j]["model"][key], or None
    when the C gather cannot vouch for every tensor (not fp32 / contiguous /
    on the model's CUDA device / the parameter's element count) -- the
    caller's per-tensor path then diagnoses or widens exactly as before."""
    if not keys:
        return None
    dev = ws[0].device
    if dev.type != "cuda":
        return None
    table = np.empty((len(keys), len(received)), dtype=np.uint64)
    status = _host_tables.gather_peer_table(received, keys, [w.numel() for w in ws], dev.index, table)
    return table if status == 0 else None


def _checked_update(j, key, w, u):
    if u.device != w.device:
        raise RuntimeError(f"Expected all tensors to be on the same device, but found at least "
                           f"two devices, {w.device} and {u.device}! (update {j}, key {key})")
    if u.numel() != w.numel():
        raise RuntimeError(f"update {j} key {key}: {tuple(u.shape)} does not match {tuple(w.shape)}")
    if u.dtype != torch.float32:
        if u.dtype == torch.float64 or u.is_complex():
            # the reference's in-place `acc += u` (:28) adds in float64 and rounds
            # once; casting u to fp32 first would round twice (1-ulp differences)
            raise TypeError(f"update {j} key {key} is {u.dtype}; p2pdl_amd aggregates float32 "
                            f"updates (fp16 / bf16 / integer updates are widened exactly)")
        u = u.to(torch.float32)  # exact widening: what the reference's add computes in
    return u.contiguous()


def _slab_fast_path(st, keys, ws, received, rule, lr, trim_frac) -> bool:
    """Updates landed by node.inbox.DeviceInbox (frozen LandedUpdate dicts
    whose fp32 tensors are rows of one device slab): the kernel table comes
    from (slab, rows, key offsets) in one broadcast -- no per-tensor Python
    work for the L x K update tensors.  Returns False (general path, with the
    reference's error behaviour) unless every condition holds: all updates
    from one inbox, every model key a slab entry of every update, model
    tensors fp32 contiguous on the slab's device with the slab layout's
    element counts (decided once per (model state, inbox) when ``st``, the
    validated model_state cache entry, is given)."""
    if not received:
        return False
    first = received[0].get("model") if isinstance(received[0], dict) else None
    if not isinstance(first, LandedUpdate):
        return False
    inbox = first.inbox
    need = st.keyset if st is not None else frozenset(keys)
    for rm in received:
        u = rm.get("model") if isinstance(rm, dict) else None
        if not isinstance(u, LandedUpdate) or u.inbox is not inbox or not u.slab_keys >= need:
            return False
    cached = st.extra.get("slab") if st is not None else None
    if cached is not None and cached[0]() is inbox:  # a weak reference: the cache keeps no inbox alive
        offsets = cached[1]
    else:
        layout, dev = inbox.layout, inbox.slab.device
        offsets = []
        for key, t in zip(keys, ws):
            off, _, n = layout[key]
            if t.dtype != torch.float32 or t.device != dev or not t.is_contiguous() or t.numel() != n:
                return False
            offsets.append(off)
        offsets = tuple(offsets)
        if st is not None:
            st.extra["slab"] = (weakref.ref(inbox), offsets)
    rows = tuple(rm["model"].row for rm in received)
    # the launch itself is cached on the validated model-state entry: the same
    # rows, rule and trim as the last call over this inbox -> the same device
    # table, launched again with no per-call work (ops.relaunch)
    ck = (rows, rule, trim_frac)
    last = st.extra.get("launch") if st is not None else None
    # ordered after land()'s row copies (they ran on the listener threads'
    # streams), and the next round's land() into these rows after this kernel
    with inbox.consuming():
        if last is not None and last[0] == ck and last[1]() is inbox:
            ops.relaunch(last[2], inbox.slab.device, len(ws), len(rows), lr)
        else:
            entry = ops.aggregate_slab_rows_(ws, inbox.slab, rows, offsets, rule, lr=lr, trim_frac=trim_frac,
                                             w_ptrs=st.ptrs if st is not None else None,
                                             numels=st.numels if st is not None else None)
            if st is not None and entry is not None:
                st.extra["launch"] = (ck, weakref.ref(inbox), entry)
    return True


def _consuming(received):
    """General path over landed updates (e.g. mixed with plain dicts): the
    launch in this block is ordered after each inbox's landing copies and
    registered with it before it is queued (DeviceInbox.consuming)."""
    inboxes = {}
    for rm in received:
        u = rm.get("model") if isinstance(rm, dict) else None
        if isinstance(u, LandedUpdate):
            inboxes[id(u.inbox)] = u.inbox
    if not inboxes:
        return _NO_INBOX
    if len(inboxes) == 1:
        return next(iter(inboxes.values())).consuming()
    stack = contextlib.ExitStack()
    try:
        for inbox in inboxes.values():
            stack.enter_context(inbox.consuming())
    except BaseException:
        stack.close()  # release the locks already taken
        raise
    return stack


_NO_INBOX = contextlib.nullcontext()


def broadcast_global_model_update(self):
    """Behaviour of reference aggregation.py:66-77 (networking is out of
    scope): pickle the state_dict, one TCP connection per neighbour, 4-byte
    big-endian length prefix.  The envelope is node.envelope's: each fp32
    weight lands by DMA in a pinned slot laid out as torch's storage blob and
    the socket sends it from there; receivers see the same keys and values
    (the reference receiver only calls load_state_dict, node/node.py:242-244).
    A message over 2**32-1 bytes cannot be framed by the 4-byte prefix: the
    reference fails inside to_bytes; this raises a clear error first."""
    with envelope.LOCK:  # the parts alias the envelope's pinned buffer until sent
        parts = envelope.envelope_parts(self.model.state_dict(), self.addr, self.port)
        msg_len = sum(p.nbytes for p in parts)
        if msg_len > 0xFFFFFFFF:
            raise OverflowError(f"global model message of {msg_len} bytes exceeds the 4-byte length prefix")
        for neighbor in self.neighbors:
            with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
                s.connect((neighbor.addr, neighbor.port))
                s.sendall(msg_len.to_bytes(4, byteorder="big"))
                for p in parts:  # the weights straight from the DMA target
                    s.sendall(p)
                logging.debug(f"Broadcasted global model update to {neighbor.addr}:{neighbor.port}")
