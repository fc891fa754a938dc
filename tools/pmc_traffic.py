#!/usr/bin/env python3
"""OUT_DIR/traffic_<workload>.json (then copied to profiles/) from the FETCH_SIZE / WRITE_SIZE passes of a GPU session
(tools/gpu_session_r02.sh): HBM-side bytes of the largest k_bdpt_sample dispatch, i.e. one
bench-sized launch of the workload (tools/prof_render.py). FETCH_SIZE / WRITE_SIZE are in KB
(MI355X_MICROARCH.md, HBM section). The guide's x2 FETCH correction is calibrated for 16-B/lane
streaming reads only; this kernel's memory-side reads are gathers (BVH nodes, primitives), scratch
(path vertices, spilled registers) and frame atomics, so the raw value is reported as traffic and the
x2 figure as an upper bound.
usage: pmc_traffic.py OUT_DIR WORKLOAD_KEY "description" [kernel_stats.csv]"""
import csv
import glob
import json
import os
import sys


def biggest(d, counter):
    best = None
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_bdpt_sample" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                v = float(r["Counter_Value"])
                if best is None or v > best[0]:
                    best = (v, r["Kernel_Name"], int(r["Grid_Size"]))
    return best


def main():
    out, key, desc = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch = biggest(os.path.join(out, "pmc_fetch"), "FETCH_SIZE")
    write = biggest(os.path.join(out, "pmc_write"), "WRITE_SIZE")
    if fetch is None or write is None:
        sys.exit("no k_bdpt_sample FETCH_SIZE / WRITE_SIZE rows found under " + out)
    rec = {
        "workload": desc,
        "workload_key": key,
        "kernel": fetch[1],
        "fetch_kb": fetch[0], "write_kb": write[0],
        "hbm_read_bytes": fetch[0] * 1024, "hbm_write_bytes": write[0] * 1024,
        "hbm_bytes_per_launch": (fetch[0] + write[0]) * 1024,
        "hbm_read_bytes_x2_upper": 2 * fetch[0] * 1024,
        "note": "FETCH_SIZE/WRITE_SIZE in KB, one launch, separate --pmc passes; x2 FETCH correction "
                "(16-B streaming reads) not applied",
    }
    if len(sys.argv) > 4 and os.path.exists(sys.argv[4]):   # the same launch's duration, kernel trace
        for r in csv.DictReader(open(sys.argv[4])):
            if r["Name"] == fetch[1]:
                rec["kernel_ms"] = float(r["AverageNs"]) / 1e6
    path = os.path.join(out, f"traffic_{key}.json")   # copied into profiles/ after the session
    with open(path, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
