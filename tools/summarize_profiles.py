#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh output directory into profiles/<tag>_*.{txt,json}.

For each config: the rocprofv3 kernel stats (average duration per kernel), and the HBM
traffic per launch of the dominant kernel from the PMC passes:
  traffic = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024
(gfx950: FETCH_SIZE reports half the bytes of a wide streaming read, MI355X_MICROARCH.md
section HBM; WRITE_SIZE is exact for these stores).  Writes profiles/traffic_<config>.json
which bench.py reports as roofline.traffic."""
import csv
import glob
import json
import sys
from pathlib import Path

src, tag = Path(sys.argv[1]), sys.argv[2]
dst = Path(__file__).resolve().parents[1] / "profiles"
dst.mkdir(exist_ok=True)
summary = {}
for cfg in ("fixed32", "csr", "fixed4096"):
    stats = list(glob.glob(str(src / cfg / "*kernel_stats.csv")))
    if not stats:
        continue
    rows = list(csv.DictReader(open(stats[0])))
    rows = [r for r in rows if "synth" not in r["Name"]]
    top = max(rows, key=lambda r: float(r["TotalDurationNs"]))
    (dst / f"{tag}_{cfg}_kernel_stats.csv").write_text(open(stats[0]).read())
    pmc = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(str(src / f"{cfg}_{c}" / "*counter_collection.csv"))
        if not f:
            continue
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f[0]))
                if r["Counter_Name"] == c and r["Kernel_Name"].startswith(top["Name"].split("(")[0])]
        if vals:
            pmc[c] = sum(vals) / len(vals)
    traffic = None
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        traffic = int(2 * pmc["FETCH_SIZE"] * 1024 + pmc["WRITE_SIZE"] * 1024)
        (dst / f"traffic_{cfg}.json").write_text(json.dumps({
            "kernel": top["Name"], "hbm_bytes_per_launch": traffic, "FETCH_SIZE_kB": pmc["FETCH_SIZE"],
            "WRITE_SIZE_kB": pmc["WRITE_SIZE"], "formula": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950)",
            "source": f"profiles/{tag}_{cfg}_kernel_stats.csv + rocprofv3 --pmc passes", "round": tag}, indent=1))
    summary[cfg] = {"kernel": top["Name"], "calls": int(top["Calls"]), "avg_ns": float(top["AverageNs"]),
                    "min_ns": float(top["MinNs"]), "max_ns": float(top["MaxNs"]), "pmc_kB": pmc,
                    "hbm_bytes_per_launch": traffic}
for cfg in ("fixed32", "csr", "fixed4096"):
    b = src / f"bench_{cfg}.out"
    if b.exists() and b.read_text().strip():
        summary.setdefault(cfg, {})["bench"] = json.loads(b.read_text().strip().splitlines()[-1])
(dst / f"{tag}_summary.json").write_text(json.dumps(summary, indent=1))
print(json.dumps({k: {kk: v[kk] for kk in ("avg_ns", "hbm_bytes_per_launch") if kk in v} for k, v in summary.items()},
                 indent=1))
