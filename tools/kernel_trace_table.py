"""Average duration (us) per kernel name over the last N dispatches of each, from a
rocprofv3 kernel trace csv.   python tools/kernel_trace_table.py TRACE.csv REGEX [N]"""
import collections
import csv
import re
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if re.search(sys.argv[2], r["Kernel_Name"])]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 10
by = collections.defaultdict(list)
for r in rows:
    by[r["Kernel_Name"][:90]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in by.items():
    v = v[-n:]
    print(f"{sum(v) / len(v):10.2f} us  (n={len(v)})  {k}")
