"""Host-side profile of the cfg1 drop-in call (MNIST MLP x 3 landed updates):
where the ~80 us of host work per aggregate_models call goes."""
import cProfile
import os
import pstats
import sys
import time
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from p2pdl_amd import ops  # noqa: E402
from p2pdl_amd.aggregator import aggregation as agg  # noqa: E402
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


for _ in range(50):
    call()
torch.cuda.synchronize()
N = 2000
t0 = time.perf_counter()
for _ in range(N):
    call()
torch.cuda.synchronize()
print(f"wall per call: {(time.perf_counter() - t0) / N * 1e6:.1f} us")
pr = cProfile.Profile()
pr.enable()
for _ in range(N):
    call()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
