"""Per-kernel PMC table from rocprofv3 --pmc passes (counter_collection.csv files under
the given directories): for every kernel whose name matches REGEX, each counter averaged
over that kernel's dispatches, plus derived waves/SIMD-style ratios.

    python tools/kernel_pmc_table.py REGEX DIR [DIR ...]
"""
import collections
import csv
import glob
import re
import sys


def main():
    rx = re.compile(sys.argv[1])
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[2:]:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            per = collections.defaultdict(float)
            names = {}
            for r in csv.DictReader(open(f)):
                if not rx.search(r["Kernel_Name"]):
                    continue
                k = (r["Dispatch_Id"], r["Counter_Name"])
                per[k] += float(r["Counter_Value"])
                names[r["Dispatch_Id"]] = re.sub(r"^_ZN3k2h12_GLOBAL__N_1\d+", "", r["Kernel_Name"])[:40]
            for (disp, ctr), v in per.items():
                acc[names[disp]][ctr].append(v)
    kernels = sorted(acc)
    ctrs = sorted({c for k in kernels for c in acc[k]})
    print(f"{'counter':28s}" + "".join(f"{k[:22]:>24s}" for k in kernels))
    for c in ctrs:
        vals = []
        for k in kernels:
            v = acc[k].get(c)
            vals.append(f"{sum(v) / len(v):24.4g}" if v else f"{'-':>24s}")
        print(f"{c:28s}" + "".join(vals))
    for k in kernels:
        a = {c: sum(v) / len(v) for c, v in acc[k].items()}
        if a.get("SQ_WAVES"):
            w = a["SQ_WAVES"]
            extra = [f"VALU/wave {a.get('SQ_INSTS_VALU', 0) / w:.0f}", f"SALU/wave {a.get('SQ_INSTS_SALU', 0) / w:.0f}",
                     f"LDS/wave {a.get('SQ_INSTS_LDS', 0) / w:.0f}"]
            if a.get("SQ_WAVE_CYCLES"):
                extra.append(f"wait_any_frac {a.get('SQ_WAIT_ANY', 0) / a['SQ_WAVE_CYCLES']:.3f}")
                extra.append(f"active_valu_frac {a.get('SQ_ACTIVE_INST_VALU', 0) / a['SQ_WAVE_CYCLES']:.3f}")
            if a.get("SQ_BUSY_CYCLES"):
                extra.append(f"waves/SIMD~ {a.get('SQ_WAVE_CYCLES', 0) / a['SQ_BUSY_CYCLES'] / 4 / 256:.2f}")
            print(f"{k}: " + ", ".join(extra))


if __name__ == "__main__":
    main()
