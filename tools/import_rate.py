"""Rate of the k2himport prehash paths: a synthetic TSV of N records (keys
8-64 B, values 0-200 B) resident in HBM -> k2h_amd_import_scan_device + k2h_amd_import_prehash,
against the host scan (k2h_import.cc) + pinned-staged host prehash of the same file.

    python tools/import_rate.py [--records N] [--reps R] > gpurun_out/import_rate.json
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from k2hash_amd import archive  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 23)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    rng = np.random.default_rng(1)
    n = a.records
    kl = rng.integers(8, 65, n)
    vl = rng.integers(0, 201, n)
    off = np.concatenate([[0], np.cumsum(kl + vl + 2)])
    data = rng.integers(32, 127, int(off[-1]), dtype=np.uint8)
    data[off[:-1] + kl] = 9
    data[off[1:] - 1] = 10
    size = data.size
    dev = torch.device("cuda", 0)
    f = torch.from_numpy(data).to(dev)
    torch.cuda.synchronize()

    def device_pass():
        recs = archive.import_scan_device(f)
        h1, h2 = archive.import_prehash_device(f, recs)
        return recs, h1, h2

    for _ in range(2):
        device_pass()
    torch.cuda.synchronize()
    ts, tp = [], []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        recs = archive.import_scan_device(f)  # synchronises
        t1 = time.perf_counter()
        archive.import_prehash_device(f, recs)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ts.append(t1 - t0)
        tp.append(t2 - t1)
    assert recs.shape[0] == n
    scan_s, pre_s = float(np.median(ts)), float(np.median(tp))
    tf = []
    for _ in range(a.reps + 1):
        t0 = time.perf_counter()
        archive.import_scan_prehash_device(f)
        torch.cuda.synchronize()
        tf.append(time.perf_counter() - t0)
    fused_s = float(np.median(tf[1:]))

    t0 = time.perf_counter()
    host = archive.import_scan(data)
    t1 = time.perf_counter()
    archive.import_prehash(data, host)
    t2 = time.perf_counter()
    print(json.dumps({
        "workload": f"{n} TSV records, keys 8-64 B, values 0-200 B, {size} bytes",
        "device": {"scan_s": scan_s, "prehash_s": pre_s, "records_per_s": n / (scan_s + pre_s),
                   "file_GB_per_s": size / (scan_s + pre_s) / 1e9, "scan_file_GB_per_s": size / scan_s / 1e9},
        "device_fused": {"s": fused_s, "records_per_s": n / fused_s, "file_GB_per_s": size / fused_s / 1e9},
        "host": {"scan_s": t1 - t0, "prehash_s": t2 - t1, "records_per_s": n / (t2 - t0),
                 "file_GB_per_s": size / (t2 - t0) / 1e9, "scan_threads": 1},
    }))


if __name__ == "__main__":
    main()
