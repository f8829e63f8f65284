"""Drop-in for the trainer-side local update of reference ``node/node.py``.

Reference ``Node.send_model_to_testers`` (node/node.py:265-282) builds the
update it sends as::

    current = self.model.state_dict()
    if self.previous_model_state is None:            # :272-275 first round
        local_update = {k: current[k] for k in current}
    else:                                            # :276-279
        local_update = {k: current[k] - self.previous_model_state[k] ...}
    self.previous_model_state = {k: v.clone() ...}   # :282

i.e. one subtraction and one clone kernel per key (2L launches, 20 B of
traffic per coordinate).  ``compute_local_update(self)`` returns the same
dict with every float32 tensor produced by ONE launch of the gfx950 K4
kernel (include/p2pdl.h ``p2p_delta_snapshot_segments_f32``: 16 B per
coordinate) and keeps ``self.previous_model_state`` a {key: tensor} dict as
the reference does -- its tensors are reused in place round after round.
Non-float32 entries (e.g. BatchNorm's int64 ``num_batches_tracked``) keep the
reference's own torch ops; they are a few bytes.

A maintainer replaces node/node.py:267-282 with
``local_update = compute_local_update(self)``; the pickling and sending that
follow (:284-297) are unchanged.
"""
from __future__ import annotations

import torch

from .. import ops


def compute_local_update(self) -> dict:
    current = self.model.state_dict()
    prev = getattr(self, "previous_model_state", None)
    first = prev is None
    keys = list(current.keys())
    local_update = {}
    new_prev = {}
    curs, prevs, deltas = [], [], []
    for key in keys:
        c = current[key]
        if c.dtype == torch.float32 and c.is_cuda and c.is_contiguous():
            p = None if first else prev[key]  # KeyError like :279 on a missing key
            if p is None or p.dtype != torch.float32 or p.shape != c.shape or p.device != c.device \
                    or not p.is_contiguous():
                p = torch.empty_like(c)
                if not first:  # reference semantics for an odd previous tensor: subtract it
                    p.copy_(prev[key])
            d = torch.empty_like(c)
            curs.append(c)
            prevs.append(p)
            deltas.append(d)
            local_update[key] = d
            new_prev[key] = p
        else:  # reference ops, unchanged (:275, :279, :282)
            local_update[key] = c if first else c - prev[key]
            new_prev[key] = c.clone()
    ops.delta_snapshot_segments_(curs, prevs, deltas, first=first)
    self.previous_model_state = new_prev
    return local_update
