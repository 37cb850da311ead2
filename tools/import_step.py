"""Driver for profiling bench.py's import secondary (k2himport TSV scan + prehash of an
8M-record file in HBM): builds bench.import_workload, warms up for ~150 ms, then runs
--calls calls of archive.import_scan_prehash_device.

    rocprofv3 ... -- python3 tools/import_step.py [--calls K]
"""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import bench  # noqa: E402
from k2hash_amd import archive  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    data = bench.import_workload(dev)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.15:
        archive.import_scan_prehash_device(data)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.calls):
        archive.import_scan_prehash_device(data)
    torch.cuda.synchronize()
    print(f"{(time.perf_counter() - t0) / a.calls * 1e3:.3f} ms per call")


if __name__ == "__main__":
    main()
