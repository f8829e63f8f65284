"""Probe: the reference's FedAvg ops on float16 / bfloat16 GPU tensors --
which roundings does torch-ROCm actually perform?  Compares the live result
with the restatements: every op in fp32 then rounded ("double"), or the
products (acc * fl(1/K), lr * acc) rounded once from the exact value
("fused", as v_fma_mixlo_f16 does).  Measurement tool, not product."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402

dev = torch.device("cuda", 0)
n = 535818
for dt, tdt in (("float16", torch.float16), ("bfloat16", torch.bfloat16)):
    for K in (3, 7, 10):
        w = oracle.round_16(oracle.synth_np(n, 0x5EED1601 + K, 0xFFFFF, 5e-2), dt)
        peers = [oracle.round_16(oracle.synth_np(n, 0x5EED1601 + K, p, 1e-2), dt) for p in range(K)]
        t = lambda b: torch.from_numpy(b.view(np.int16).copy()).view(tdt).to(dev)
        acc = torch.zeros(n, dtype=tdt, device=dev)
        for p in peers:
            acc += t(p)
        s_live = acc.view(torch.int16).cpu().numpy().view(np.uint16).copy()
        acc /= K
        m_live = acc.view(torch.int16).cpu().numpy().view(np.uint16).copy()
        tt = 0.1 * acc
        t_live = tt.view(torch.int16).cpu().numpy().view(np.uint16).copy()
        wt = t(w)
        wt += tt
        w_live = wt.view(torch.int16).cpu().numpy().view(np.uint16)
        f = lambda b: oracle.to_f32_16(b, dt)
        # sums
        s = np.zeros(n, np.float32)
        for p in peers:
            s = f(oracle.round_16(s + f(p), dt))
        inv = np.float32(1.0) / np.float32(K)
        m_double = oracle.round_16(s * inv, dt)
        m_fused = (oracle.round_16_once(s.astype(np.float64) * np.float64(inv), dt) if dt == "float16" else None)
        m_true = oracle.round_16(s / np.float32(K), dt)
        print(dt, K, "sum ok", np.array_equal(oracle.round_16(s, dt), s_live),
              "| m double", np.count_nonzero(m_double != m_live), "fused",
              None if m_fused is None else np.count_nonzero(m_fused != m_live), "truediv", np.count_nonzero(m_true != m_live))
        t_double = oracle.round_16(np.float32(0.1) * f(m_live), dt)
        t_fused = (oracle.round_16_once(f(m_live).astype(np.float64) * np.float64(np.float32(0.1)), dt)
                   if dt == "float16" else None)
        if dt == "float16":
            md = f(m_live).astype(np.float64)
            cand = {
                "f16(f32(0.1d*m))": oracle.round_16((np.float64(0.1) * md).astype(np.float32), dt),
                "f16once(0.1d*m)": oracle.round_16_once(np.float64(0.1) * md, dt),
                "f16(f32(f32(0.1d)*m))": oracle.round_16((np.float64(np.float32(0.1)) * md).astype(np.float32), dt),
            }
            print("   candidates:", {k: int(np.count_nonzero(v != t_live)) for k, v in cand.items()})
            for i in np.nonzero(t_double != t_live)[0][:4]:
                print(f"     i={i} m={md[i]!r} ({hex(m_live[i])}) 0.1f*m={float(np.float32(0.1) * np.float32(md[i]))!r} "
                      f"live={float(f(t_live[i:i+1])[0])!r} ({hex(t_live[i])}) double={float(f(t_double[i:i+1])[0])!r} "
                      f"({hex(t_double[i])})")
        print("   t double", np.count_nonzero(t_double != t_live), "fused",
              None if t_fused is None else np.count_nonzero(t_fused != t_live),
              "| w", np.count_nonzero(oracle.round_16(f(w) + f(t_live), dt) != w_live))
