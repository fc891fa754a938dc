#!/usr/bin/env python3
"""OUT_DIR/traffic_<workload>.json (then copied to profiles/) from the FETCH_SIZE / WRITE_SIZE passes of a GPU session
(tools/gpu_session_r03.sh): HBM-side bytes of the largest k_bdpt_sample dispatch, i.e. one
bench-sized launch of the workload (tools/prof_render.py), and that dispatch's duration from the
kernel trace collected in the same rocprofv3 run (--pmc with --kernel-trace), so the bytes are tied
to a measured kernel time. FETCH_SIZE / WRITE_SIZE are in KB (MI355X_MICROARCH.md, HBM section).
FETCH_SIZE counts half of the bytes a read moves for every access width this kernel uses — 16-B
and 4-B lane-interleaved streams, 16-B gathers at random lines (64 B per 128-B line) — and
WRITE_SIZE counts 4-B stores exactly (tools/fetch_calib.hip, profiles/r03_fetch_calibration.log),
so the HBM-side bytes of a launch are 2 x FETCH_SIZE + WRITE_SIZE.
usage: pmc_traffic.py OUT_DIR WORKLOAD_KEY "description" """
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
                    best = (v, r["Kernel_Name"], r.get("Dispatch_Id"))
    return best


def dispatch_ms(d, kernel, dispatch):
    """Duration of that dispatch in the same run's kernel trace (None without one)."""
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Kernel_Name") == kernel and (dispatch is None or r.get("Dispatch_Id") == dispatch):
                return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    return None


def main():
    out, key, desc = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch = biggest(os.path.join(out, "pmc_fetch"), "FETCH_SIZE")
    write = biggest(os.path.join(out, "pmc_write"), "WRITE_SIZE")
    if fetch is None or write is None:
        sys.exit("no k_bdpt_sample FETCH_SIZE / WRITE_SIZE rows found under " + out)
    fms = dispatch_ms(os.path.join(out, "pmc_fetch"), fetch[1], fetch[2])
    wms = dispatch_ms(os.path.join(out, "pmc_write"), write[1], write[2])
    rec = {
        "workload": desc,
        "workload_key": key,
        "kernel": fetch[1],
        "fetch_kb": fetch[0], "write_kb": write[0],
        "hbm_read_bytes": 2 * fetch[0] * 1024, "hbm_write_bytes": write[0] * 1024,
        "hbm_bytes_per_launch": (2 * fetch[0] + write[0]) * 1024,
        "fetch_pass_kernel_ms": fms, "write_pass_kernel_ms": wms,
        "kernel_ms": (fms + wms) / 2 if fms and wms else None,
        "note": "FETCH_SIZE/WRITE_SIZE in KB, one launch, separate --pmc passes each with its own kernel "
                "trace (kernel_ms = mean of the two dispatch durations); read bytes = 2 x FETCH_SIZE "
                "(calibrated: profiles/r03_fetch_calibration.log)",
    }
    path = os.path.join(out, f"traffic_{key}.json")   # copied into profiles/ after the session
    with open(path, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
