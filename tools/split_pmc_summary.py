#!/usr/bin/env python3
"""Per-variant SQ counters of tools/split_fixed_lab under rocprofv3 --pmc
(round 6): for each kernel instantiation, counters
averaged over its dispatches and the derived shares -- wait cycles per
wave-cycle (SQ_WAIT_ANY / SQ_WAVE_CYCLES), instruction-issue share
(SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES), and GRBM_GUI_ACTIVE per dispatch.
usage: split_pmc_summary.py <rocprofv3 -d dir> [out.json]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    per = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "split" not in name:
            continue
        per[(name, r["Dispatch_Id"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    agg = defaultdict(lambda: defaultdict(list))
    for (name, _), ctrs in per.items():
        for c, v in ctrs.items():
            agg[name][c].append(sum(v))
    out = {}
    for name, ctrs in agg.items():
        m = {c: sum(v) / len(v) for c, v in ctrs.items()}
        wc = m.get("SQ_WAVE_CYCLES") or 1.0
        short = name.split("(")[0]
        out[short] = {"dispatches": len(next(iter(ctrs.values()))), **{c: round(v, 1) for c, v in m.items()},
                      "wait_share": round(m.get("SQ_WAIT_ANY", 0) / wc, 4),
                      "wait_inst_share": round(m.get("SQ_WAIT_INST_ANY", 0) / wc, 4),
                      "issue_share": round(m.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4),
                      "wave_cycles_per_wave": round(wc / max(m.get("SQ_WAVES", 1), 1), 1)}
    js = json.dumps(out, indent=1)
    print(js)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(js + "\n")


if __name__ == "__main__":
    main()
