#!/usr/bin/env python3
"""Average each PMC counter per dispatch of the kernels matching a regex, over all
pmc pass directories under a root.  usage: pmc_summary.py <root> [kernel-regex]"""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1]
rx = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if rx.search(r["Kernel_Name"]):
            name = r["Kernel_Name"].split("(")[0][-60:]
            agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in agg.items():
    print(f"== {name}")
    for c in sorted(cs):
        v = cs[c]
        print(f"   {c:32s} n={len(v):3d} mean={sum(v)/len(v):.6g}")
