#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh output directory into profiles/<tag>_*.

For each config: the rocprofv3 kernel stats; the TIMED WINDOW of the dominant kernel (its
last `steps` dispatches in the kernel trace -- the bench's timed region, after the
clock-ramp warm-up), which is what the bench line's roofline.achieved uses; and from the
PMC passes, per launch of that kernel:
  traffic = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024
(gfx950: FETCH_SIZE reports half the bytes of a wide streaming read, MI355X_MICROARCH.md
section HBM; WRITE_SIZE is exact for these stores) -> profiles/traffic_<config>.json, and
SQ_INSTS_VALU -> profiles/valu_<config>.json (bench.py's roofline.traffic / valu_frac).

usage: summarize_profiles.py <profile dir> <tag>"""
import csv
import glob
import json
import sys
from pathlib import Path

src, tag = Path(sys.argv[1]), sys.argv[2]
dst = Path(__file__).resolve().parents[1] / "profiles"
dst.mkdir(exist_ok=True)
summary = {}
for d in sorted(p for p in src.iterdir() if p.is_dir() and "_pmc" not in p.name):
    cfg = d.name
    stats = glob.glob(str(d / "**" / "*kernel_stats.csv"), recursive=True)
    trace = glob.glob(str(d / "**" / "*kernel_trace.csv"), recursive=True)
    bench = src / f"bench_{cfg}.out"
    line = json.loads(bench.read_text().strip().splitlines()[-1]) if bench.exists() and bench.read_text().strip() else None
    if not stats or not trace:
        continue
    want = "ralledata" if cfg == "ralledata" else "fnv_"  # the config's dominant product kernel
    rows = [r for r in csv.DictReader(open(stats[0])) if "synth" not in r["Name"] and want in r["Name"]]
    top = max(rows, key=lambda r: float(r["TotalDurationNs"]))
    (dst / f"{tag}_{cfg}_kernel_stats.csv").write_text(open(stats[0]).read())
    disp = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(trace[0]))
                  if r["Kernel_Name"] == top["Name"])
    steps = line["steps"] if line else 0
    win = disp[-steps:] if steps else disp
    durs = [e - s for s, e in win]
    window = {"kernel": top["Name"], "dispatches_total": len(disp), "window_dispatches": len(win),
              "window_avg_ns": sum(durs) / len(durs), "window_min_ns": min(durs), "window_max_ns": max(durs),
              "window_span_ns_first_start_to_last_end": win[-1][1] - win[0][0],
              "all_dispatches_avg_ns": float(top["AverageNs"])}
    pmc = {}
    for f in glob.glob(str(src / f"{cfg}_pmc*" / "**" / "*counter_collection.csv"), recursive=True):
        per = {}  # dispatch -> counter -> sum over XCDs / SEs
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].split("(")[0] == top["Name"].split("(")[0]:
                d = per.setdefault(r["Dispatch_Id"], {})
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        last = sorted(per, key=int)[-10:]  # the timed dispatches of the (warmed) PMC run
        for d in last:
            for c, v in per[d].items():
                pmc.setdefault(c, []).append(v)
    pmc = {k: sum(v) / len(v) for k, v in pmc.items()}
    traffic = None
    # keys (records) per launch of the profiled kernel: bench.py scales the per-launch counts
    # to other launch sizes by it
    keys = (line or {}).get("config", {}).get("keys_per_gpu")
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        traffic = int(2 * pmc["FETCH_SIZE"] * 1024 + pmc["WRITE_SIZE"] * 1024)
        (dst / f"traffic_{cfg}.json").write_text(json.dumps({
            "kernel": top["Name"], "hbm_bytes_per_launch": traffic, "FETCH_SIZE_kB": pmc["FETCH_SIZE"],
            "WRITE_SIZE_kB": pmc["WRITE_SIZE"], "formula": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950)",
            "source": f"profiles/{tag}_{cfg}_summary.json (rocprofv3 --pmc passes)", "round": tag,
            "written_by": "tools/summarize_profiles.py over tools/profile_round.sh (tools/gpu/final.sh)",
            "keys_per_launch": keys}, indent=1))
    if "SQ_INSTS_VALU" in pmc:
        (dst / f"valu_{cfg}.json").write_text(json.dumps({
            "kernel": top["Name"], "valu_insts_per_launch": pmc["SQ_INSTS_VALU"],
            "salu_insts_per_launch": pmc.get("SQ_INSTS_SALU"), "lds_insts_per_launch": pmc.get("SQ_INSTS_LDS"),
            "waves_per_launch": pmc.get("SQ_WAVES"),
            "source": f"profiles/{tag}_{cfg}_summary.json (rocprofv3 --pmc SQ_INSTS_VALU pass)", "round": tag,
            "written_by": "tools/summarize_profiles.py over tools/profile_round.sh (tools/gpu/final.sh)",
            "keys_per_launch": keys}, indent=1))
    s = {"window": window, "pmc_per_launch": pmc, "hbm_bytes_per_launch": traffic}
    if line:
        kern_ms = line["kernel_ms"]
        s["bench"] = {k: line.get(k) for k in ("value", "ms_per_step", "kernel_ms", "roofline")}
        s["window_vs_bench_event_time"] = window["window_avg_ns"] / 1e6 / kern_ms
    (dst / f"{tag}_{cfg}_summary.json").write_text(json.dumps(s, indent=1))
    summary[cfg] = {"window_avg_us": window["window_avg_ns"] / 1e3, "traffic": traffic,
                    "valu_insts": pmc.get("SQ_INSTS_VALU"),
                    "window_vs_bench": s.get("window_vs_bench_event_time")}
print(json.dumps(summary, indent=1))
