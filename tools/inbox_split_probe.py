import time, pickle, torch, sys
sys.path.insert(0, '.')
import bench
from p2pdl_amd.node.inbox import ZeroCopyParser, DeviceInbox
dev = torch.device('cuda', 0)
shapes = bench.resnet18_param_shapes()
ser = [pickle.dumps({k: torch.randn(s) for k, s in shapes}) for _ in range(16)]
n = len(ser[0])
pin = [torch.empty(n, dtype=torch.uint8, pin_memory=True) for _ in ser]
for p, s in zip(pin, ser):
    p.copy_(torch.frombuffer(bytearray(s), dtype=torch.uint8))
d = torch.empty(n, dtype=torch.uint8, device=dev)
for rep in range(3):
    torch.cuda.synchronize(); t = time.perf_counter()
    for p in pin:
        d.copy_(p, non_blocking=True)
    torch.cuda.synchronize(); t_dma = time.perf_counter() - t
    t = time.perf_counter()
    for s in ser:
        ZeroCopyParser(s).parse()
    t_parse = time.perf_counter() - t
print(f"16 x {n/1e6:.1f} MB: H2D from pinned {t_dma*1e3:.1f} ms ({16*n/t_dma/1e9:.1f} GB/s); parse {t_parse*1e3:.1f} ms")
template = {k: torch.empty(s, device=dev) for k, s in shapes}
inbox = DeviceInbox(template, k_max=16, device=dev)
msgs = [inbox.message_buffer(n) for _ in ser]
for m, s in zip(msgs, ser):
    m.buf[:n].copy_(torch.frombuffer(bytearray(s), dtype=torch.uint8))
for rep in range(3):
    inbox.reset(); torch.cuda.synchronize(); t = time.perf_counter()
    for m in msgs:
        inbox.land(m)
    t_host = time.perf_counter() - t
    torch.cuda.synchronize(); t_all = time.perf_counter() - t
print(f"land pinned: host loop {t_host*1e3:.1f} ms, with device drain {t_all*1e3:.1f} ms")
