#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes of tools/bin/fetch_calib (tools/fetch_calib.hip), plus
# the raw request counters behind FETCH_SIZE (TCC_BUBBLE = 128-B requests, TCC_EA0_RDREQ,
# TCC_EA0_RDREQ_32B) and each kernel's duration from the kernel trace.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-calib}
mkdir -p $OUT
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE "TCC_BUBBLE_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  n=${c%% *}
  timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/$n -o run -- tools/bin/fetch_calib > $OUT/$n.log 2>&1 || { echo "STOP $c"; tail -5 $OUT/$n.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, re
out = sys.argv[1]
req, lines = {}, {}
for l in open(f"{out}/FETCH_SIZE.log"):
    m = re.match(r"(k_\w+) (?:requested|written)_bytes (\d+)(?: lines (\d+))?", l)
    if m:
        req[m.group(1)] = int(m.group(2))
        if m.group(3): lines[m.group(1)] = int(m.group(3))
lines.setdefault("k_gather16", 64 << 20)
name = lambda k: {"k_gather_n<4>": "k_gather64", "k_gather_n<8>": "k_gather128"}.get(k, k)
dur = {}
for f in glob.glob(f"{out}/FETCH_SIZE/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = name(re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", ""))
        dur[k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
for n in ("FETCH_SIZE", "WRITE_SIZE", "TCC_BUBBLE_sum"):
    for f in glob.glob(f"{out}/{n}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = name(re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", ""))
            if k not in req: continue
            v = float(r["Counter_Value"])
            if r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE"):
                b = v * 1024
                print(f"{r['Counter_Name']:10s} {k:12s} counter_bytes {b:.4g} requested {req[k]:.4g} ratio {b / req[k]:.4f}")
            else:
                print(f"{r['Counter_Name']:22s} {k:12s} {v:.4g}" + (f" per line {v / lines[k]:.3f}" if k in lines else ""))
for k, t in sorted(dur.items()):
    msg = f"duration {k:12s} {t * 1e3:.3f} ms"
    if k in lines:
        msg += f"; if 128 B move per line: {lines[k] * 128 / t / 1e12:.2f} TB/s, if 64 B: {lines[k] * 64 / t / 1e12:.2f} TB/s"
    print(msg)
PY
