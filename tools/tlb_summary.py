#!/usr/bin/env python3
"""Translation (UTCL1) counters of tools/lib_pair_ab.py's rowsclone case
under rocprofv3 --pmc (round 6): per launch, the rows kernel over the slab,
the chunk list over .clone()d dicts and over the slab's own views.  The
chunk-kernel dispatches are told apart by the case's fixed order: one setup
launch over the clones, one over the views, (since the case compares builds)
one bit-check launch over the clones per build, then per rep [clones, views]
(even reps) or [views, clones] (odd).  SETUP: the chunk launches before the
reps -- 3 for one build (2 for the tool as profiles/r06/tlb/tlb_p*.json ran
it).  Measurement tool, not product.
usage: tlb_summary.py <rocprofv3 output dir> [out.json] [SETUP=3]"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    files = glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit("no counter_collection.csv")
    disp = collections.OrderedDict()
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "fedavg_split_kernel" not in name:
                continue
            d = disp.setdefault(int(r["Dispatch_Id"]), {"kernel": name, "c": {}})
            d["c"][r["Counter_Name"]] = d["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    rows, chunks = [], []
    for i in sorted(disp):
        (rows if "false, 2," in disp[i]["kernel"] else chunks).append(disp[i]["c"])
    setup = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    labels = []
    for rep in range((len(chunks) - setup) // 2):
        labels += ["clones", "views"] if rep % 2 == 0 else ["views", "clones"]
    groups = {"rows (slab)": rows[1:], "chunks (clones)": [], "chunks (slab views)": []}
    for lab, c in zip(labels, chunks[setup:]):
        groups["chunks (clones)" if lab == "clones" else "chunks (slab views)"].append(c)
    out = {}
    for g, cs in groups.items():
        keys = sorted({k for c in cs for k in c})
        out[g] = {k: sum(c.get(k, 0.0) for c in cs) / max(len(cs), 1) for k in keys}
        out[g]["launches"] = len(cs)
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
