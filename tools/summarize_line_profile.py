#!/usr/bin/env python3
"""Recompute every bench-line figure from the profile of the same run.

Input: a tools/profile_line.sh directory -- the driver's command (python bench.py) under
rocprofv3 --kernel-trace --marker-trace, with bench.py's roctx ranges "timed:<label>"
around the synchronised timed region of the headline and of each secondary.

For each label: the kernels that ran inside its range; the dominant product kernel (largest
total time, synthetic-input kernels excluded); its dispatch count (must equal the entry's
`steps`) and average duration (the "window"); the HBM fraction recomputed from it with the
line's own algorithmic bytes per launch, beside the line's `roofline.frac`.  The k2himport
entries time whole calls (three kernels and a host sync each), so their window is the
range's span / steps and their per-call kernel sum is listed too.

  python tools/summarize_line_profile.py <dir> <tag> [out.json]   -> profiles/<tag>_line_summary.json
"""
import csv
import glob
import json
import sys
from pathlib import Path

HBM_PEAK = 8.0e12
WALL_TIMED = ("import", "import_mdbm")  # the line's roofline for these uses the call's wall time


def _rows(pattern, src):
    files = glob.glob(str(src / "**" / pattern), recursive=True)
    return list(csv.DictReader(open(files[0]))) if files else []


def ranges(src):
    """[(label, start_ns, end_ns)] of the roctx ranges named timed:<label>."""
    out = []
    for r in _rows("*marker_api_trace.csv", src):
        text = next((v for v in r.values() if isinstance(v, str) and v.startswith("timed:")), None)
        if text:
            out.append((text.split(":", 1)[1], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return sorted(out, key=lambda x: x[1])


def main():
    src, tag = Path(sys.argv[1]), sys.argv[2]
    line = json.loads((src / "bench_line.json").read_text().strip().splitlines()[-1])
    kern = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
            for r in _rows("*kernel_trace.csv", src)]
    entries = {"headline": line, **(line.get("secondary") or {})}
    out = {"tag": tag, "command": "python bench.py (the driver's default) under rocprofv3 --kernel-trace "
                                  "--marker-trace (tools/profile_line.sh)",
           "how": "frac_profile = the line's algorithmic bytes per launch / window / 8 TB/s; window = the dominant "
                  "kernel's average duration inside the entry's roctx range (import entries: range span / steps)",
           "entries": {}}
    for label, s, e in ranges(src):
        ent = entries.get(label)
        if ent is None or "roofline" not in ent:
            continue
        inside = [k for k in kern if k[1] >= s and k[2] <= e and "synth" not in k[0]]
        by = {}
        for name, a, b in inside:
            by.setdefault(name, []).append(b - a)
        steps = ent.get("steps")
        rf = ent["roofline"]
        algo = rf["algorithmic_bytes_per_launch"]
        rec = {"steps": steps, "range_span_ms": (e - s) / 1e6, "line_frac": rf["frac"],
               "line_ms_per_step": ent.get("ms_per_step"), "line_kernel_ms": ent.get("kernel_ms"),
               "kernels": {n: {"dispatches": len(d), "avg_us": sum(d) / len(d) / 1e3} for n, d in by.items()}}
        if label in WALL_TIMED:
            per_call = (e - s) / steps
            rec["window_us"] = per_call / 1e3
            rec["kernel_sum_per_call_us"] = sum(sum(d) for d in by.values()) / steps / 1e3
        else:
            top = max(by, key=lambda n: sum(by[n]))
            rec["dominant"] = top
            rec["dispatches_ok"] = len(by[top]) == steps
            rec["window_us"] = sum(by[top]) / len(by[top]) / 1e3
        rec["frac_profile"] = algo / (rec["window_us"] * 1e-6) / HBM_PEAK
        rec["frac_profile_over_line"] = rec["frac_profile"] / rf["frac"]
        out["entries"][label] = rec
    dst = Path(sys.argv[3]) if len(sys.argv) > 3 else \
        Path(__file__).resolve().parents[1] / "profiles" / f"{tag}_line_summary.json"
    dst.write_text(json.dumps(out, indent=1) + "\n")
    for k, v in out["entries"].items():
        print(f"{k:15s} window {v['window_us']:9.1f} us  frac profile {v['frac_profile']:.3f}  "
              f"line {v['line_frac']:.3f}  ratio {v['frac_profile_over_line']:.3f}  "
              f"{'' if v.get('dispatches_ok', True) else 'DISPATCH COUNT != steps'}")
    missing = [k for k, v in entries.items() if "roofline" in v and k not in out["entries"]]
    if missing:
        print("no range for:", missing)


if __name__ == "__main__":
    main()
