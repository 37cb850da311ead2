#!/usr/bin/env python3
"""Table of PMC counters per variant from an output directory of the round-2 tools/pmc_variants.sh (at commit f74668a):
per-dispatch sums over XCDs, median over dispatches of the hash kernel, plus the derived
clock (GRBM_GUI_ACTIVE per XCD / duration) and VALU issue utilisation
(SQ_INSTS_VALU x 4.19 cycles / (SIMDs x cycles)).   usage: pmc_table.py <dir> [kernel-substring]"""
import collections
import csv
import glob
import statistics
import sys

root = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "fnv_"
res = collections.defaultdict(dict)
for f in glob.glob(f"{root}/*/pmc_counter_collection.csv"):
    v = f.split("/")[-2].split("_")[0]
    acc = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"] and "ring_list" not in r["Kernel_Name"]:
            acc[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    per = collections.defaultdict(list)
    for (d, c), val in acc.items():
        per[c].append(val)
    for c, vals in per.items():
        res[v][c] = statistics.median(vals)
    t = f.replace("counter_collection", "kernel_trace")
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(t))
            if sub in r["Kernel_Name"] and "ring_list" not in r["Kernel_Name"]]
    if durs:
        res[v].setdefault("dur_ns", statistics.median(durs))
for v, d in res.items():
    if "GRBM_GUI_ACTIVE" in d:
        d["clock_GHz"] = d["GRBM_GUI_ACTIVE"] / 8 / d["dur_ns"]
        if "SQ_INSTS_VALU" in d:
            d["valu_util"] = d["SQ_INSTS_VALU"] * 4.19 / (1024 * d["GRBM_GUI_ACTIVE"] / 8)
    if "SQ_WAVE_CYCLES" in d and "GRBM_GUI_ACTIVE" in d:
        d["waves_per_simd"] = d["SQ_WAVE_CYCLES"] * 4 / (1024 * d["GRBM_GUI_ACTIVE"] / 8)
    if "SQ_WAIT_ANY" in d and "SQ_WAVE_CYCLES" in d:
        d["wait_any_frac"] = d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"]
keys = sorted({k for d in res.values() for k in d})
print("counter".ljust(24), *[v.rjust(12) for v in sorted(res)])
for k in keys:
    print(k.ljust(24), *[f"{res[v].get(k, 0):12.4g}" for v in sorted(res)])
