#!/usr/bin/env python3
"""Summarise a rocprofv3 output directory (SQLite run_results.db or the CSV
files of --output-format csv) for committing under profiles/.

usage: rocpd_summary.py <rocprofv3 -d dir> [kernel-substring]
Prints the kernel stats (calls, average / min / max ns) and, for a --pmc run,
every counter averaged per dispatch of the kernels matching the substring,
plus the derived figures used in DESIGN.md (effective clock from
GRBM_GUI_ACTIVE, VALU issue share, wait share)."""
import csv
import glob
import json
import os
import sqlite3
import sys
from collections import defaultdict


def rows_db(path):
    c = sqlite3.connect(path)
    disp = {}
    for r in c.execute("select dispatch_id, name, start, end from kernels"):
        disp[r[0]] = (r[1], r[3] - r[2])
    ctr = defaultdict(lambda: defaultdict(float))
    try:
        for did, kname, name, val in c.execute(
                "select dispatch_id, kernel_name, counter_name, value from counters_collection"):
            ctr[(did, kname)][name] += val
    except sqlite3.OperationalError:
        pass
    return disp, ctr


def rows_csv(d):
    disp, ctr = {}, defaultdict(lambda: defaultdict(float))
    for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            disp[(fn, r["Dispatch_Id"])] = (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            ctr[((fn, r["Dispatch_Id"]), r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    return disp, ctr


def main():
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    disp, ctr = rows_db(dbs[0]) if dbs else rows_csv(d)
    stats = defaultdict(list)
    for kname, dur in disp.values():
        stats[kname].append(dur)
    out = {"kernels": []}
    for k, v in sorted(stats.items(), key=lambda kv: -sum(kv[1])):
        out["kernels"].append({"name": k, "calls": len(v), "avg_ns": sum(v) / len(v), "min_ns": min(v),
                               "max_ns": max(v), "total_ns": sum(v)})
    per = defaultdict(list)
    for (did, kname), cs in ctr.items():
        if sub in kname:
            per[kname].append(cs)
    for kname, lst in per.items():
        names = sorted(set().union(*lst))
        avg = {n: sum(x.get(n, 0.0) for x in lst) / len(lst) for n in names}
        rec = {"kernel": kname, "dispatches": len(lst), "counters_avg": avg}
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
                if n in avg:
                    rec[f"{n}/SQ_WAVE_CYCLES"] = avg[n] / wc
        if "SQ_INSTS_VALU" in avg and "SQ_WAVES" in avg:
            rec["valu_insts_per_wave"] = avg["SQ_INSTS_VALU"] / avg["SQ_WAVES"]
        dur = [x["avg_ns"] for x in out["kernels"] if x["name"] == kname]
        if "GRBM_GUI_ACTIVE" in avg and dur:
            rec["effective_clock_ghz"] = avg["GRBM_GUI_ACTIVE"] / 8 / dur[0]
        out.setdefault("pmc", []).append(rec)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
