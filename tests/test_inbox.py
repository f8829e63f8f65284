"""Receive / deserialize path: p2pdl_amd.node.inbox.

CPU tests pin the restricted parser to pickle.loads on torch-produced
pickles of the reference's message shapes (node/node.py:285 pickles a
state_dict of the models/model.py MLP); GPU tests land updates in the device
slab and aggregate them through the drop-in."""
import os
import pickle
import socket
import threading
import types

import numpy as np
import pytest
import torch

import oracle
from helpers import assert_bits_equal
from p2pdl_amd.node.inbox import DeviceInbox, UpdateParser, ZeroCopyParser, recv_message

MLP_SHAPES = [("fc1.weight", (512, 784)), ("fc1.bias", (512,)), ("fc2.weight", (256, 512)),
              ("fc2.bias", (256,)), ("fc3.weight", (10, 256)), ("fc3.bias", (10,))]  # models/model.py:6-8


def mlp_update(seed):
    out = {}
    for i, (k, s) in enumerate(MLP_SHAPES):
        out[k] = torch.from_numpy(oracle.synth(int(np.prod(s)), seed, i, 1e-2).reshape(s))
    return out


def same(raw, ref):
    assert list(raw) == list(ref)
    for k in ref:
        a = np.ascontiguousarray(raw[k].array()).reshape(-1)
        r = ref[k].contiguous().numpy().reshape(-1)
        assert raw[k].size == tuple(ref[k].shape), k
        assert a.dtype == r.dtype and np.array_equal(a.view(np.uint8), r.view(np.uint8)), k


PARSERS = [UpdateParser.parse, lambda d: ZeroCopyParser(d).parse()]


@pytest.mark.parametrize("parse", PARSERS, ids=["c-unpickler", "zero-copy"])
def test_parser_matches_pickle_loads_mlp_update(parse):
    upd = mlp_update(1)
    data = pickle.dumps(upd)  # reference node/node.py:285
    same(parse(data), pickle.loads(data))


@pytest.mark.parametrize("proto", [3, 4, 5])
@pytest.mark.parametrize("parse", PARSERS, ids=["c-unpickler", "zero-copy"])
def test_parser_batchnorm_scalars_views_and_ordereddict(parse, proto):
    net = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.BatchNorm1d(5))
    sd = net.state_dict()  # OrderedDict incl. an int64 0-d buffer
    sd["view.t"] = torch.arange(12, dtype=torch.float32).reshape(3, 4).t()  # strided view
    sd["view.slice"] = torch.arange(20, dtype=torch.float32)[5:9]           # storage offset
    sd["x" * 300] = torch.ones(3)                                           # BINUNICODE key
    data = pickle.dumps(sd, protocol=proto)
    same(parse(data), pickle.loads(data))


def test_zero_copy_parser_payloads_alias_the_message():
    data = bytearray(pickle.dumps({"w": torch.arange(1000, dtype=torch.float32)}))
    raw = ZeroCopyParser(data).parse()
    arr = raw["w"].array()
    assert arr[7] == 7.0
    i = bytes(data).index(np.arange(1000, dtype=np.float32)[5:9].tobytes())
    data[i:i + 4] = np.float32(-1).tobytes()  # mutate the message: the view sees it
    assert raw["w"].array()[5] == -1.0


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned",))


@pytest.mark.parametrize("payload", [
    {"a": _Evil()},
    {"a": torch.ones(2), "b": _Evil()},
    [torch.ones(3)],                       # not a dict of tensors
    {"a": 3},
])
def test_parser_rejects_anything_but_tensors(payload):
    for parse in PARSERS:
        with pytest.raises(pickle.UnpicklingError):
            parse(pickle.dumps(payload))


def test_zero_copy_parser_rejects_protocol_2_and_truncation():
    with pytest.raises(pickle.UnpicklingError):
        ZeroCopyParser(pickle.dumps({"a": torch.ones(2)}, protocol=2)).parse()
    data = pickle.dumps({"a": torch.ones(2)})
    with pytest.raises((pickle.UnpicklingError, IndexError, ValueError)):
        ZeroCopyParser(data[:-20]).parse()


def test_recv_message_framing_and_early_close():
    a, b = socket.socketpair()
    msg = pickle.dumps({"type": "model_update", "model": pickle.dumps(mlp_update(2)), "addr": "x", "port": 1})

    def send():
        b.sendall(len(msg).to_bytes(4, "big"))
        for i in range(0, len(msg), 4096):  # the reference's 4 KiB pieces
            b.sendall(msg[i:i + 4096])
        b.sendall((1000).to_bytes(4, "big") + b"short")  # a truncated second message
        b.close()

    th = threading.Thread(target=send)
    th.start()
    got = recv_message(a)
    assert bytes(got) == msg
    assert recv_message(a) is None  # peer closed early: dropped, like node/node.py:111
    th.join()
    a.close()


@pytest.mark.gpu
def test_device_inbox_lands_bit_exact_and_aggregates(cuda, monkeypatch):
    from p2pdl_amd.aggregator import aggregation as agg

    monkeypatch.setattr(agg, "broadcast_global_model_update", lambda self: None)
    k = 5
    template = {name: torch.zeros(s, device=cuda) for name, s in MLP_SHAPES}
    inbox = DeviceInbox(template, k_max=8, device=cuda)
    ser = [pickle.dumps(mlp_update(10 + j)) for j in range(k)]
    landed = [inbox.land(s) for s in ser]
    torch.cuda.synchronize()
    for s, got in zip(ser, landed):
        ref = pickle.loads(s)
        assert list(got) == list(ref)
        for key in ref:
            assert got[key].is_cuda and got[key].shape == ref[key].shape
            assert_bits_equal(got[key].cpu().numpy(), ref[key].numpy(), what=key)
    # the landed views feed the drop-in unchanged (node/node.py:138 -> :316)
    n = sum(int(np.prod(s)) for _, s in MLP_SHAPES)
    w = oracle.synth(n, 3, 0xFFFFF, 5e-2)
    model = torch.nn.Module()
    offs = 0
    for name, s in MLP_SHAPES:
        m = int(np.prod(s))
        mod, attr = name.split(".")
        if not hasattr(model, mod):
            model.add_module(mod, torch.nn.Module())
        getattr(model, mod).register_parameter(attr, torch.nn.Parameter(
            torch.from_numpy(w[offs:offs + m].reshape(s).copy()).to(cuda)))
        offs += m
    node = types.SimpleNamespace(model=model, trainers_list=[0] * k, addr="a", port=1, neighbors=[],
                                 received_models=[{"model": u, "sender": j} for j, u in enumerate(landed)])
    agg.aggregate_models(node)
    got = np.concatenate([t.detach().cpu().numpy().reshape(-1) for t in model.state_dict().values()])
    flat = [np.concatenate([pickle.loads(s)[name].numpy().reshape(-1) for name, _ in MLP_SHAPES]) for s in ser]
    want, _ = oracle.fedavg(flat, w)
    assert_bits_equal(got, want, what="fedavg over landed updates")


@pytest.mark.gpu
def test_device_inbox_parses_cuda_pickles(cuda):
    upd = {k: v.to(cuda) for k, v in mlp_update(4).items()}
    data = pickle.dumps(upd)  # a CUDA sender's bytes (storage location 'cuda:0')
    inbox = DeviceInbox({k: v for k, v in upd.items()}, k_max=1, device=cuda)
    got = inbox.land(data, 0)
    torch.cuda.synchronize()
    for key in upd:
        assert torch.equal(got[key], upd[key]), key


@pytest.mark.gpu
def test_broadcast_from_gpu_model_one_transfer(cuda):
    """the GPU model's broadcast carries the same
    keys/values (bit-exact) with the reference framing."""
    import socket as sk

    from p2pdl_amd.aggregator import aggregation as agg

    net = torch.nn.Sequential(torch.nn.Linear(33, 64), torch.nn.BatchNorm1d(64), torch.nn.Linear(64, 10)).to(cuda)
    srv = sk.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    got = {}

    def serve():
        c, _ = srv.accept()
        got["msg"] = pickle.loads(bytes(recv_message(c)))
        c.close()

    th = threading.Thread(target=serve)
    th.start()
    nd = types.SimpleNamespace(model=net, addr="127.0.0.1", port=9,
                               neighbors=[types.SimpleNamespace(addr="127.0.0.1", port=srv.getsockname()[1])])
    agg.broadcast_global_model_update(nd)
    th.join(10)
    srv.close()
    msg = got["msg"]
    assert msg["type"] == "global_model_update" and msg["addr"] == "127.0.0.1" and msg["port"] == 9
    ref = net.state_dict()
    assert list(msg["model"]) == list(ref)
    for k, v in ref.items():
        assert torch.equal(msg["model"][k], v.cpu()), k
        assert msg["model"][k].untyped_storage().nbytes() == v.numel() * v.element_size(), k
