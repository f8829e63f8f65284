#!/usr/bin/env python3
"""Lab (round 5): one FedAvg workload of K rows x C coordinates at a given
row pitch, three launches -- the unit a rocprofv3 --pmc pass profiles (UTCL1
translation counters vs the rows' address span).  usage:
python tools/span_pmc.py C pitch [K]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2pdl_amd import ops  # noqa: E402


def main():
    C, pitch = int(sys.argv[1]), int(sys.argv[2])
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    dev = torch.device("cuda", 0)
    slab = torch.empty((K, pitch), dtype=torch.float32, device=dev)
    for p in range(K):
        ops.fill_synthetic_(slab[p, :C], 0x5EED0002, p, 1e-2)
    table = ops.pointer_table([slab[p, :C] for p in range(K)], dev)
    w = torch.empty(C, dtype=torch.float32, device=dev)
    ops.fill_synthetic_(w, 0x5EED0002, 0xFFFFF, 5e-2)
    for _ in range(3):
        ops.aggregate(None, "fedavg", w=w, lr=0.1, table=table)
    torch.cuda.synchronize()
    print(f"done C={C} pitch={pitch} K={K}")


if __name__ == "__main__":
    main()
