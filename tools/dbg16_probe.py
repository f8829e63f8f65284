import numpy as np, torch, sys
sys.path.insert(0, "/root/repo")
import oracle
from p2pdl_amd import ops
dev = torch.device("cuda", 0)
n, k = 200000, 3
for dt, tdt in (("float16", torch.float16), ("bfloat16", torch.bfloat16)):
    w = oracle.round_16(oracle.synth_np(n, 0x5EED1601, 0xFFFFF, 5e-2), dt)
    peers = [oracle.round_16(oracle.synth_np(n, 0x5EED1601, p, 1e-2), dt) for p in range(k)]
    wt = torch.from_numpy(w.view(np.int16).copy()).view(tdt).to(dev)
    ops.fedavg16_apply_(wt, [torch.from_numpy(p.view(np.int16).copy()).view(tdt).to(dev) for p in peers])
    got = wt.view(torch.int16).cpu().numpy().view(np.uint16)
    want = oracle.fedavg16_np(peers, w, dt)
    bad = np.nonzero(got != want)[0]
    print(dt, "mismatches", bad.size)
    for i in bad[:6]:
        f = lambda b: float(oracle.to_f32_16(np.array([b], np.uint16), dt)[0])
        acc = 0.0
        print(i, "w", f(w[i]), "peers", [f(p[i]) for p in peers], "got", f(got[i]), hex(got[i]), "want", f(want[i]), hex(want[i]))
