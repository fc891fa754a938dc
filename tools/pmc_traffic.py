#!/usr/bin/env python3
"""profiles/traffic_<tag>.json from the FETCH_SIZE / WRITE_SIZE passes of tools/gpu_session.sh:
HBM-side bytes of the largest k_bdpt_sample dispatch (one bench-sized launch, CBspheres 480x360
128 spp m5). FETCH_SIZE/WRITE_SIZE are in KB (MI355X_MICROARCH.md, HBM section). The guide's x2
FETCH correction is calibrated for 16-B/lane streaming reads only; this kernel's memory-side reads
are mostly scratch (register spills, path vertices) and frame atomics, so the raw value is
reported as traffic and the x2 figure as an upper bound.
usage: pmc_traffic.py OUT_DIR TAG"""
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
    out, tag = sys.argv[1], sys.argv[2]
    fetch = biggest(os.path.join(out, "pmc_fetch"), "FETCH_SIZE")
    write = biggest(os.path.join(out, "pmc_write"), "WRITE_SIZE")
    rec = {
        "workload": "CBspheres 480x360 s128 m5, one launch (tools/prof_render.py)",
        "kernel": fetch[1],
        "fetch_kb": fetch[0], "write_kb": write[0],
        "hbm_read_bytes": fetch[0] * 1024, "hbm_write_bytes": write[0] * 1024,
        "hbm_bytes_per_launch": (fetch[0] + write[0]) * 1024,
        "hbm_read_bytes_x2_upper": 2 * fetch[0] * 1024,
        "note": "FETCH_SIZE/WRITE_SIZE in KB; x2 FETCH correction (16-B streaming reads) not applied",
    }
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                        f"traffic_{tag}.json")
    with open(path, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
