#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter_collection.csv files per kernel name (all dispatches).
usage: pmc_summary.py DIR [DIR ...] -> table of counters per kernel."""
import collections
import csv
import glob
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("bdpt::", "")
            k = re.sub(r"\(.*", "", k).replace("void ", "")
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, cs in sorted(acc.items()):
    if k.startswith("__amd"):
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"    {c:26s} {v:12.4g}")
