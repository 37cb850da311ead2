"""Summarise tools/gpu/import_prof.sh (rocprofv3 over tools/import_step.py): per call of
k2h_amd_import_scan_prehash_device, the kernel time and the PMC counters summed over its
kernels (tsv_a, tsv_b; round-3 trees before r03i also the block-function scan and
tsv_count), averaged over the last
calls -> profiles/traffic_import.json, profiles/valu_import.json (bench.py's
secondary.import roofline) and profiles/<tag>_import_summary.json.

    python tools/summarize_import_profile.py gpurun_out/prof_import r02ar
    python tools/summarize_import_profile.py gpurun_out/prof_import_mdbm r06k import_mdbm
(the mdbm form: tools/gpu/import_prof.sh with MDBM=1 -> profiles/traffic_import_mdbm.json,
valu_import_mdbm.json, bench.py's secondary.import_mdbm roofline)
"""
import collections
import csv
import glob
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
OURS = ("tsv_a_kernel", "tsv_count_kernel", "tsv_b_kernel", "tsv_scan_kernel", "ROCPRIM_400200")  # rocprim 4.2: our scan


def ours(name):
    return any(k in name for k in OURS)


def main():
    src, tag = Path(sys.argv[1]), sys.argv[2]
    name = sys.argv[3] if len(sys.argv) > 3 else "import"
    prof = ROOT / "profiles"
    # kernel time per call from the trace: the last 10 calls' dispatches of our kernels
    rows = [r for r in csv.DictReader(open(src / "trace" / "run_kernel_trace.csv")) if ours(r["Kernel_Name"])]
    walks = [i for i, r in enumerate(rows) if "tsv_b_kernel" in r["Kernel_Name"]]
    calls = 10
    first = walks[-calls - 1] + 1
    per = collections.defaultdict(float)
    for r in rows[first:]:
        nm = r["Kernel_Name"]
        key = next((k for k in OURS[:4] if k in nm), "lookback_scan" if "lookback" in nm else "rocprim_scan")
        per[key] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / calls
    gpu_us = sum(per.values()) / 1e3
    shutil.copy(src / "trace" / "run_kernel_stats.csv", prof / f"{tag}_{name}_kernel_stats.csv")
    # PMC: per counter, summed over our kernels, averaged over the calls of each pass
    pmc = {}
    for p in sorted(src.glob("pmc*")):
        fs = glob.glob(str(p / "**" / "*counter_collection.csv"), recursive=True)
        if not fs:
            continue
        crow = [r for r in csv.DictReader(open(fs[0])) if ours(r["Kernel_Name"])]
        ncalls = len({r["Dispatch_Id"] for r in crow if "tsv_b_kernel" in r["Kernel_Name"]})
        acc = collections.defaultdict(float)
        for r in crow:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
        for k, v in acc.items():
            pmc[k] = v / ncalls
    traffic = int(2 * pmc["FETCH_SIZE"] * 1024 + pmc["WRITE_SIZE"] * 1024)
    kern = " + ".join(sorted(per)) + " (one call)"
    (prof / f"traffic_{name}.json").write_text(json.dumps({
        "kernel": kern, "hbm_bytes_per_launch": traffic, "FETCH_SIZE_kB": pmc["FETCH_SIZE"],
        "WRITE_SIZE_kB": pmc["WRITE_SIZE"], "formula": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950)",
        "round": tag, "keys_per_launch": 1 << 23,
        "written_by": "tools/summarize_import_profile.py over tools/gpu/import_prof.sh"}, indent=1) + "\n")
    (prof / f"valu_{name}.json").write_text(json.dumps({
        "kernel": kern, "valu_insts_per_launch": pmc["SQ_INSTS_VALU"], "salu_insts_per_launch": pmc.get("SQ_INSTS_SALU"),
        "lds_insts_per_launch": pmc.get("SQ_INSTS_LDS"), "round": tag, "keys_per_launch": 1 << 23,
        "written_by": "tools/summarize_import_profile.py over tools/gpu/import_prof.sh"}, indent=1) + "\n")
    s = {"per_kernel_us_per_call": {k: v / 1e3 for k, v in per.items()}, "gpu_us_per_call": gpu_us,
         "pmc_per_call": pmc, "hbm_bytes_per_call": traffic,
         "source": "tools/gpu/import_prof.sh: rocprofv3 over tools/import_step.py (8M records, 1.16 GB, "
                   + ("mdbm" if name == "import_mdbm" else "TSV") + ")"}
    (prof / f"{tag}_{name}_summary.json").write_text(json.dumps(s, indent=1) + "\n")
    print(json.dumps(s, indent=1))


if __name__ == "__main__":
    main()
