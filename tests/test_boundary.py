"""Host-side boundary behaviour of the drop-in (CPU; no kernel launches)."""
import pickle
import socket
import threading
import time
import types

import pytest
import torch

from helpers import load_golden
from p2pdl_amd import ops
from p2pdl_amd import _native as N
from p2pdl_amd.aggregator import aggregation as agg
from p2pdl_amd.utils.waiting import wait_for_models

META, _ = load_golden()


def node(model, updates, trainers=None):
    return types.SimpleNamespace(model=model, trainers_list=[0] * (len(updates) if trainers is None else trainers),
                                 received_models=[{"model": u, "sender": i} for i, u in enumerate(updates)],
                                 addr="127.0.0.1", port=7000, neighbors=[])


def test_zero_updates_returns_none_without_clear(monkeypatch):
    calls = []
    monkeypatch.setattr(agg, "broadcast_global_model_update", lambda s: calls.append(s))
    m = torch.nn.Linear(3, 2)
    before = {k: v.clone() for k, v in m.state_dict().items()}
    nd = node(m, [], trainers=0)
    inbox = nd.received_models
    assert agg.aggregate_models(nd) is None
    assert nd.received_models is inbox and calls == []
    assert all(torch.equal(before[k], v) for k, v in m.state_dict().items())
    assert META["behaviour"]["k0"]["returns"] == "None"


def test_missing_key_raises_keyerror_like_reference():
    m = torch.nn.Linear(3, 2)
    nd = node(m, [{"weight": torch.zeros(2, 3)}])
    with pytest.raises(KeyError) as e:
        agg.aggregate_models(nd)
    assert e.value.args[0] == "bias"  # the reference raises KeyError(<missing key>) too
    assert META["behaviour"]["missing_key"]["raises"] == "KeyError"
    assert len(nd.received_models) == 1


def test_integer_buffer_raises_reference_runtime_error():
    m = torch.nn.BatchNorm1d(4)  # num_batches_tracked is int64
    upd = {k: torch.ones_like(v) for k, v in m.state_dict().items()}
    nd = node(m, [upd])
    with pytest.raises(RuntimeError) as e:
        agg.aggregate_models(nd)
    assert str(e.value) == META["behaviour"]["int_buffer"]["message"]
    assert len(nd.received_models) == 1  # not cleared, like the reference


def test_cpu_tensors_fail_loudly_no_fallback():
    m = torch.nn.Linear(3, 2)
    nd = node(m, [{k: torch.ones_like(v) for k, v in m.state_dict().items()}])
    with pytest.raises((N.NativeUnavailable, RuntimeError)):
        agg.aggregate_models(nd)
    with pytest.raises((N.NativeUnavailable, RuntimeError)):
        ops.median([torch.zeros(8), torch.ones(8)])


def test_rule_and_trim_helpers():
    assert ops.rule_id("fedavg") == 0 and ops.rule_id("median") == 1 and ops.rule_id("trimmed") == 2
    with pytest.raises(ValueError):
        ops.rule_id("krum")
    assert [ops.trim_count(k) for k in (1, 5, 10, 128, 256)] == [0, 1, 2, 25, 51]
    with pytest.raises(ValueError):
        ops.trim_count(4, 0.5)


def test_wait_for_models_semantics():
    inbox = []
    assert wait_for_models(inbox, 0) is True
    t = threading.Timer(0.05, lambda: inbox.extend([1, 2]))
    t.start()
    assert wait_for_models(inbox, 2, timeout=5, poll=0.01) is True
    assert wait_for_models([], 1, timeout=0.05, poll=0.01) is False


def test_broadcast_framing_matches_reference():
    """4-byte big-endian length + pickle body, one connection per neighbour
    (reference aggregation.py:66-77)."""
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]
    got = {}

    def serve():
        c, _ = srv.accept()
        n = int.from_bytes(c.recv(4), "big")
        buf = b""
        while len(buf) < n:
            buf += c.recv(65536)
        got["msg"] = pickle.loads(buf)
        c.close()

    th = threading.Thread(target=serve)
    th.start()
    m = torch.nn.Linear(2, 1)
    nd = types.SimpleNamespace(model=m, addr="127.0.0.1", port=9,
                               neighbors=[types.SimpleNamespace(addr="127.0.0.1", port=port)])
    agg.broadcast_global_model_update(nd)
    th.join(5)
    srv.close()
    assert got["msg"]["type"] == "global_model_update" and got["msg"]["port"] == 9
    assert torch.equal(got["msg"]["model"]["weight"], m.state_dict()["weight"])


def test_pack_messages_alignment():
    host, offs, lens = ops.pack_messages([b"a", b"", b"x" * 17, b"y" * 32])
    assert offs == [0, 16, 32, 64] and lens == [1, 0, 17, 32]
    assert bytes(host[32:49]) == b"x" * 17
