"""Host cost of the pieces of one cfg1 drop-in call (MNIST MLP x 3 landed
updates), each timed alone over many calls: where the ~12 us go.
Measurement tool, not product."""
import logging
import os
import sys
import time
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from p2pdl_amd import _native as N  # noqa: E402
from p2pdl_amd import ops  # noqa: E402
from p2pdl_amd.aggregator import aggregation as agg  # noqa: E402
from p2pdl_amd.aggregator.model_state import model_state  # noqa: E402
from p2pdl_amd.node.inbox import DeviceInbox  # noqa: E402

dev = torch.device("cuda", 0)
shapes = [("fc1.weight", (512, 784)), ("fc1.bias", (512,)), ("fc2.weight", (256, 512)),
          ("fc2.bias", (256,)), ("fc3.weight", (10, 256)), ("fc3.bias", (10,))]
model = torch.nn.Module()
for nm, s in shapes:
    model.register_parameter(nm.replace(".", "__"), torch.nn.Parameter(torch.randn(s, device=dev) * 0.05,
                                                                        requires_grad=False))
inbox = DeviceInbox(model.state_dict(), k_max=3, device=dev)
for p in range(3):
    ops.fill_synthetic_(inbox.slab[p], 7, p, 1e-2)
landed = [inbox.view(j) for j in range(3)]
node = types.SimpleNamespace(model=model, trainers_list=[0] * 3, addr="127.0.0.1", port=1, neighbors=[],
                             received_models=[])
agg.broadcast_global_model_update = lambda self: None


def call():
    node.received_models.extend({"model": u, "sender": j} for j, u in enumerate(landed))
    agg.aggregate_models(node)


for _ in range(100):
    call()
torch.cuda.synchronize()
st = model_state(model)[2]
entry = st.extra["launch"][2]
raw = N.stream_handle(0)
L = len(shapes)
parts = {
    "whole aggregate_models call": call,
    "received_models.extend (bench side)": lambda: node.received_models.extend(
        {"model": u, "sender": j} for j, u in enumerate(landed)),
    "model_state (validate cache)": lambda: model_state(model),
    "ops.relaunch (ctypes + hip launch)": lambda: ops.relaunch(entry, dev, L, 3, 0.1),
    "_launch_table only": lambda: ops._launch_table(entry[0].data_ptr(), L, entry[1], 3, entry[2], entry[3], 0.1,
                                                    stream=raw),
    "inbox.slab_consumed (event record)": inbox.slab_consumed,
    "inbox.order_after_landing": inbox.order_after_landing,
    "N.stream_handle": lambda: N.stream_handle(0),
    "torch.cuda.current_device": torch.cuda.current_device,
    "logging.info f-string": lambda: logging.info(f"[{node.addr}:{node.port}] Model aggregation completed"),
    "logging.info lazy": lambda: logging.info("[%s:%s] Model aggregation completed", node.addr, node.port),
}
reps = 20000
for name, fn in parts.items():
    for _ in range(200):
        fn()
    node.received_models.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
        if name.startswith("received"):
            node.received_models.clear()
    torch.cuda.synchronize()
    print(f"{(time.perf_counter() - t0) / reps * 1e6:7.2f} us  {name}", flush=True)
