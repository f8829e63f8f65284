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
('fedavg' | 'median' | 'trimmed', README.md:10 "Byzantine fault" TODO),
``lr`` (:36) and ``trim_frac``.
"""
import logging
import pickle
import socket

import torch

from .. import ops
from ..utils.waiting import wait_for_models

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

    state = self.model.state_dict()
    keys = list(state.keys())
    updates = []
    for received_model in received:  # KeyError on a missing key, like :28
        local_update = received_model["model"]
        updates.append([local_update[key] for key in keys])

    for key in keys:  # the reference raises at the division for integer tensors (:32)
        t = state[key]
        if not t.is_floating_point():
            name = _TORCH_TYPE_NAMES.get(t.dtype, str(t.dtype))
            raise RuntimeError(f"result type Float can't be cast to the desired output type {name}")
        if t.dtype != torch.float32:
            raise NotImplementedError(f"p2pdl_amd aggregates float32 state_dicts; {key} is {t.dtype}")

    ws = [state[key] for key in keys]
    peer_lists = []
    for j, upd in enumerate(updates):
        row = []
        for key, w, u in zip(keys, ws, upd):
            if u.device != w.device:
                raise RuntimeError(f"Expected all tensors to be on the same device, but found at least "
                                   f"two devices, {w.device} and {u.device}! (update {j}, key {key})")
            if u.numel() != w.numel():
                raise RuntimeError(f"update {j} key {key}: {tuple(u.shape)} does not match "
                                   f"{tuple(w.shape)}")
            if u.dtype != torch.float32:
                u = u.to(torch.float32)
            row.append(u.contiguous())
        peer_lists.append(row)

    # state_dict() tensors are views of the parameters: updating them in place
    # updates the model, exactly like the reference's `+=` at :38.
    ws_c = [w if w.is_contiguous() else w.contiguous() for w in ws]
    ops.aggregate_segments_(ws_c, peer_lists, rule or AGGREGATION_RULE, lr=lr, trim_frac=trim_frac)
    for w, wc in zip(ws, ws_c):
        if wc is not w:
            w.copy_(wc)

    logging.info(f"[{self.addr}:{self.port}] Model aggregation completed, applied local updates.")

    # Clear received models for the next round (:43)
    self.received_models.clear()

    # Broadcast the newly aggregated global model (:46)
    broadcast_global_model_update(self)


def broadcast_global_model_update(self):
    """Unchanged behaviour of reference aggregation.py:66-77 (networking is out
    of scope): pickle the state_dict, one TCP connection per neighbour, 4-byte
    big-endian length prefix."""
    model_state = self.model.state_dict()
    data = pickle.dumps({"type": "global_model_update", "model": model_state,
                         "addr": self.addr, "port": self.port})
    msg_len = len(data)
    for neighbor in self.neighbors:
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            s.connect((neighbor.addr, neighbor.port))
            s.sendall(msg_len.to_bytes(4, byteorder="big"))
            s.sendall(data)
            logging.debug(f"Broadcasted global model update to {neighbor.addr}:{neighbor.port}")
