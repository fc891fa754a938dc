#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes of tools/bin/fetch_calib (tools/fetch_calib.hip).
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-calib}
mkdir -p $OUT
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/$c -o run -- tools/bin/fetch_calib > $OUT/$c.log 2>&1 || { echo "STOP $c"; tail -5 $OUT/$c.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, re
out = sys.argv[1]
req = {}
for l in open(f"{out}/FETCH_SIZE.log"):
    m = re.match(r"(k_\w+) (?:requested|written)_bytes (\d+)", l)
    if m: req[m.group(1)] = int(m.group(2))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{out}/{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
            if k in req:
                b = float(r["Counter_Value"]) * 1024
                print(f"{c:10s} {k:11s} counter_bytes {b:.4g} requested {req[k]:.4g} ratio {b / req[k]:.4f}")
PY
