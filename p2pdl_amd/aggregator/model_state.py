"""``self.model.state_dict()`` for the aggregator, without rebuilding it.

The reference reads its keys and tensors from ``self.model.state_dict()``
(aggregator/aggregation.py:15,27,37-38 -- rebuilt once per key there).  That
call walks every module and detaches every tensor: 6 us for the MNIST MLP,
~230 us for a ResNet-18 (122 entries) on a host core -- at the reference's
MLP size the whole aggregation kernel takes 5 us.  ``model_state(model)``
returns the same (keys, tensors) from a per-model cache and re-validates it
on every call against everything that could change what state_dict() would
return:

  * the module tree: every module's ``_modules`` entries are the cached
    children, and no module gained / lost a parameter, buffer or child;
  * every entry: ``owner._parameters[name]`` / ``owner._buffers[name]`` is
    still the cached object, at the cached address with the cached shape
    (a ``param.data = ...`` swap or an in-place resize moves one of them);
  * no state_dict hook, and no module whose class overrides state_dict,
    _save_to_state_dict or get_extra_state (such a model always takes the
    real state_dict(): its keys or values are the class's business).

Any mismatch rebuilds the entry from the real ``state_dict(keep_vars=True)``,
and the rebuilt walk must reproduce its keys and objects exactly, else the
model is marked uncacheable.  The returned tensors are ``detach()``-ed views
of the parameters, like state_dict()'s, so writing them updates the model
in place exactly as the reference's ``+=`` at :38 does.
"""
from __future__ import annotations

import threading
import weakref

import torch
from torch import nn

_BASE = nn.Module


def _plain_module(mod) -> bool:
    cls = type(mod)
    return (cls.state_dict is _BASE.state_dict and cls._save_to_state_dict is _BASE._save_to_state_dict
            and cls.get_extra_state is _BASE.get_extra_state and not mod._state_dict_hooks
            and not mod._state_dict_pre_hooks)


class ModelState:
    """(keys, tensors) of one model's state_dict plus what validates them."""

    __slots__ = ("keys", "tensors", "ptrs", "numels", "modules", "entries", "keyset", "extra")

    def __init__(self, keys, tensors, modules, entries):
        self.keys = keys          # state_dict key order
        self.tensors = tensors    # detached views (what state_dict() returns)
        self.ptrs = tuple(t.data_ptr() for t in tensors)
        self.numels = tuple(t.numel() for t in tensors)
        self.modules = modules    # (module, n_params, n_buffers, n_children, children tuple, npb frozenset)
        self.entries = entries    # (owner dict, name, object, data_ptr, shape)
        self.keyset = frozenset(keys)
        self.extra = {}           # per-consumer derived data (e.g. slab offsets), dies with the entry

    def valid(self) -> bool:
        for mod, np_, nb, nc, kids, npb in self.modules:
            if (len(mod._parameters) != np_ or len(mod._buffers) != nb or len(mod._modules) != nc
                    or mod._state_dict_hooks or mod._state_dict_pre_hooks
                    or mod._non_persistent_buffers_set != npb):
                return False
            for name, child in kids:
                if mod._modules.get(name) is not child:
                    return False
        for owner, name, obj, ptr, shape in self.entries:
            if owner.get(name) is not obj or obj.data_ptr() != ptr or obj.shape != shape:
                return False
        return True


_CACHE: "weakref.WeakKeyDictionary[nn.Module, ModelState | None]" = weakref.WeakKeyDictionary()
_LOCK = threading.Lock()


def _walk(mod, prefix, modules, entries, keys):
    """state_dict()'s traversal (parameters, then persistent buffers, then
    children in registration order); False if a module is not plain."""
    if not _plain_module(mod):
        return False
    kids = tuple((n, c) for n, c in mod._modules.items())
    modules.append((mod, len(mod._parameters), len(mod._buffers), len(mod._modules), kids,
                    frozenset(mod._non_persistent_buffers_set)))
    for name, p in mod._parameters.items():
        if p is not None:
            entries.append((mod._parameters, name, p, p.data_ptr(), p.shape))
            keys.append(prefix + name)
    for name, b in mod._buffers.items():
        if b is not None and name not in mod._non_persistent_buffers_set:
            entries.append((mod._buffers, name, b, b.data_ptr(), b.shape))
            keys.append(prefix + name)
    for name, child in kids:
        if child is not None and not _walk(child, prefix + name + ".", modules, entries, keys):
            return False
    return True


def _build(model) -> ModelState | None:
    modules, entries, keys = [], [], []
    if not _walk(model, "", modules, entries, keys):
        return None
    sd = model.state_dict(keep_vars=True)
    if list(sd.keys()) != keys or any(sd[k] is not e[2] for k, e in zip(keys, entries)):
        return None  # not the traversal torch itself does: never cache
    return ModelState(keys, [e[2].detach() for e in entries], modules, entries)


def model_state(model) -> tuple[list, list, ModelState | None]:
    """(keys, tensors, cache entry or None) equal to
    ``list(model.state_dict().items())`` unzipped."""
    try:
        st = _CACHE.get(model, False)
    except TypeError:  # not weak-referenceable
        st = None
    if st is not False and st is not None and st.valid():
        return st.keys, st.tensors, st
    if st is None:  # known uncacheable
        sd = model.state_dict()
        return list(sd.keys()), list(sd.values()), None
    st = _build(model)
    with _LOCK:
        try:
            _CACHE[model] = st
        except TypeError:
            pass
    if st is None:
        sd = model.state_dict()
        return list(sd.keys()), list(sd.values()), None
    return st.keys, st.tensors, st
