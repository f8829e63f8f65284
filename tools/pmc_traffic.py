#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per launch.

Usage: pmc_traffic.py <fetch_dir> <write_dir> <kernel-substring> <workload>
                      <coords_per_launch> <peers> [out.json]

Each pass is its own rocprofv3 run (FETCH_SIZE takes 3 TCC slots, WRITE_SIZE
2; they do not fit one pass).  Corrections follow
/opt/skills/guides/MI355X_MICROARCH.md §HBM: both counters are in KiB;
on gfx950 FETCH_SIZE reports half of the bytes of a wide (16 B/lane)
coalesced streaming read, so it is doubled; WRITE_SIZE is exact for 16-B
streaming stores.  The result is written where bench.py picks it up
(profiles/traffic_<workload>.json) and must match the launch bench.py times.
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, kname):
    """Per-launch value of `counter` for kernel-name substring kname.  kname
    "a+b" (one aggregation call = launches of kernel a and of kernel b, e.g.
    the split FedAvg kernel and the VGPR kernel over its remainder): every
    matching dispatch is summed and divided by the dispatches of a."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    names = kname.split("+")
    vals = {}
    first = set()
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                kn = row.get("Kernel_Name", "")
                if row.get("Counter_Name") != counter or not any(x in kn for x in names):
                    continue
                key = (fn, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
                if names[0] in kn:
                    first.add(key)
    if not vals or not first:
        raise SystemExit(f"no {counter} rows for kernel '{kname}' in {d}")
    v = sorted(vals.values())
    return v, sum(v) / len(first)


def main():
    fdir, wdir, kname, workload, coords, peers = sys.argv[1:7]
    out = sys.argv[7] if len(sys.argv) > 7 else None
    coords, peers = int(coords), int(peers)
    fv, fetch_kib = per_dispatch(fdir, "FETCH_SIZE", kname)
    wv, write_kib = per_dispatch(wdir, "WRITE_SIZE", kname)
    read_b = 2 * fetch_kib * 1024  # gfx950 half-count of wide streaming reads
    write_b = write_kib * 1024
    if workload == "delta":  # read cur + prev, write delta + prev (16 B per parameter)
        alg_read, alg_write = 8 * coords, 8 * coords
    else:  # K peer reads + w read, w write
        alg_read, alg_write = 4 * coords * (peers + 1), 4 * coords
    res = {
        "workload": workload, "kernel": kname, "coords_per_launch": coords, "peers": peers,
        "dispatches": [len(fv), len(wv)],
        "fetch_size_kib_raw": fetch_kib, "write_size_kib": write_kib,
        "hbm_read_bytes_per_launch": read_b, "hbm_write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": read_b + write_b,
        "alg_bytes_per_launch": alg_read + alg_write,
        "traffic_over_alg": (read_b + write_b) / (alg_read + alg_write),
        "correction": "FETCH_SIZE x2 (gfx950 wide-read half count), KiB -> B; WRITE_SIZE exact",
    }
    js = json.dumps(res, indent=1)
    print(js)
    if out:
        with open(out, "w") as f:
            f.write(js + "\n")


if __name__ == "__main__":
    main()
