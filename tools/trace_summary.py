#!/usr/bin/env python3
"""Per-kernel, per-grid averages from a rocprofv3 --kernel-trace CSV, for
profiles/<round>/final (the numbers bench.py's HIP events must agree with).

usage: trace_summary.py <rocprofv3 -d dir> <out dir>
Writes kernel_trace_by_grid.json (calls and average duration per kernel name
and grid size) and cfg3_split_remainder_trace.json (each cfg3 plane launch:
the split kernel over whole CU rounds plus the VGPR kernel's remainder that
follows it on the stream -- their average durations and the call span)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    src, out = sys.argv[1], sys.argv[2]
    path = glob.glob(os.path.join(src, "*kernel_trace.csv"))[0]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0]
            grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, grid, r["Queue_Id"]))
    rows.sort()
    by = defaultdict(list)
    for s, e, name, grid, _ in rows:
        if "p2p::" not in name or "synth_kernel" in name or "sha256" in name:
            continue  # the product's aggregation kernels only (not torch's reference legs)
        by[f"{name} grid={grid}"].append((e - s) / 1e3)
    summary = {k: {"calls": len(v), "avg_us": round(sum(v) / len(v), 1)}
               for k, v in sorted(by.items(), key=lambda kv: -len(kv[1]) * sum(kv[1]))}
    with open(os.path.join(out, "kernel_trace_by_grid.json"), "w") as f:
        json.dump(summary, f, indent=1)
    # cfg3 planes: a split launch of the cfg3 plane's grid directly followed
    # (same queue) by the flat remainder
    pairs = []
    for i, (s, e, name, grid, q) in enumerate(rows[:-1]):
        s2, e2, name2, grid2, q2 = rows[i + 1]
        if name.endswith("fedavg_split_kernel<false, false, false>") and "fedavg_flat_kernel" in name2 and q == q2:
            pairs.append((grid, (e - s) / 1e3, (e2 - s2) / 1e3, (e2 - s) / 1e3))
    groups = defaultdict(list)
    for g, a, b, span in pairs:
        groups[g].append((a, b, span))
    res = {f"split grid={g}": {"launches": len(v),
                               "split_avg_us": round(sum(x[0] for x in v) / len(v), 1),
                               "remainder_avg_us": round(sum(x[1] for x in v) / len(v), 1),
                               "call_span_avg_us": round(sum(x[2] for x in v) / len(v), 1)}
           for g, v in groups.items()}
    with open(os.path.join(out, "cfg3_split_remainder_trace.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
