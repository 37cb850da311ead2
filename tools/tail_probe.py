#!/usr/bin/env python3
"""Wave-generation tail of the 4 KiB line-DMA kernel: per-key time of the product kernel at
key counts that fill a whole number of resident-wave generations (10 one-wave blocks per
CU x CUs x 64 keys each) versus BASELINE config 5's 1M keys (6.4 generations), interleaved
in one process.  A per-key time well below config 5's at whole generations means the
partial last generation costs time.

  python tools/tail_probe.py [--gens 4,5,6,7] [--rounds 5] [--reps 10]
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import k2hash_amd  # noqa: E402
from k2hash_amd import batch  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--gens", default="4,5,6,7")
p.add_argument("--rounds", type=int, default=5)
p.add_argument("--reps", type=int, default=10)
a = p.parse_args()
dev = torch.device("cuda:0")
L = 4096
cus = torch.cuda.get_device_properties(0).multi_processor_count
per_gen = cus * 10 * 64  # keys per generation of resident waves
counts = {"config5": 1 << 20}
for g in a.gens.split(","):
    counts[f"gen{g}"] = int(g) * per_gen
nmax = max(counts.values())
keys = batch.synth_bytes(nmax * L, dev)
out = torch.empty(nmax, dtype=torch.int64, device=dev)
times = {k: [] for k in counts}
for i in range(20):
    k2hash_amd.hash_fixed(keys[: counts["config5"] * L], L, out=(out[: counts["config5"]], None))
torch.cuda.synchronize()
for r in range(a.rounds):
    for name, n in counts.items():
        kv, ov = keys[: n * L], out[:n]
        for i in range(2):
            k2hash_amd.hash_fixed(kv, L, out=(ov, None))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(a.reps):
            k2hash_amd.hash_fixed(kv, L, out=(ov, None))
        e1.record()
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1) / a.reps)
for name, n in counts.items():
    med = statistics.median(times[name])
    print(json.dumps({"name": name, "keys": n, "generations": round(n / per_gen, 3), "ms_median": med,
                      "ns_per_key": med * 1e6 / n, "frac_8TBps": n * (L + 8) / med / 1e6 / 8000}), flush=True)
