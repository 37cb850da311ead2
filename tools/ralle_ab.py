#!/usr/bin/env python3
"""A/B timing of RALLEDATA assembly variants (lab library), interleaved rounds in one
process, on bench.py's ralledata workload (8M records, keys 8-64 B, values 0-256 B).
Every variant's blobs and blob offsets are first compared byte for byte with variant 73
(the round-1/2 group kernel).

  python tools/ralle_ab.py [--variants 73,0] [--rounds 5] [--reps 10]
"""
import argparse
import json
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
os.environ.setdefault("K2H_AMD_BATCH_LIB", str(ROOT / "tools" / "lab" / "libk2hash_amd_lab.so"))

import torch  # noqa: E402

from k2hash_amd import _native, batch, ralledata  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--variants", default="73,0")
p.add_argument("--rounds", type=int, default=5)
p.add_argument("--reps", type=int, default=10)
p.add_argument("--n", type=int, default=1 << 23)
a = p.parse_args()
dev = torch.device("cuda:0")
n = a.n
sets = []
for s in range(2):
    ko = batch.synth_offsets(n, dev, 8, 64, first_key=s * n)
    vo = batch.synth_offsets(n, dev, 0, 256, seed=batch.SEED_LENS + 7, first_key=s * n)
    kb, vb = int(ko[-1].item()), int(vo[-1].item())
    kd = batch.synth_bytes(kb, dev, byte_off=s * (1 << 36))
    vd = batch.synth_bytes(vb, dev, byte_off=s * (1 << 36) + (1 << 33))
    total = 80 * n + kb + vb
    sets.append(((kd, ko, vd, vo), torch.empty(total, dtype=torch.uint8, device=dev),
                 torch.empty(n + 1, dtype=torch.int64, device=dev), total))
algo = (kb + vb + 16 * (n + 1)) + (80 * n + kb + vb + 8 * (n + 1))


def run(i):
    (kd, ko, vd, vo), blob, boff, total = sets[i & 1]
    ralledata.build_ralledata(kd, ko, vd, vo, out=blob, blob_off=boff, total=total)


variants = [int(v) for v in a.variants.split(",")]
_native.lab_set_variant(73)
run(0)
ref_blob, ref_off = sets[0][1].clone(), sets[0][2].clone()
for v in variants:
    _native.lab_set_variant(v)
    sets[0][1].zero_()
    run(0)
    torch.cuda.synchronize()
    ok = torch.equal(sets[0][1], ref_blob) and torch.equal(sets[0][2], ref_off)
    print(f"variant {v}: parity {'OK' if ok else 'MISMATCH'}", flush=True)
    if not ok:
        sys.exit(1)
del ref_blob
_native.lab_set_variant(variants[0])
for i in range(100):
    run(i)
times = {v: [] for v in variants}
for r in range(a.rounds):
    for v in variants:
        _native.lab_set_variant(v)
        for i in range(3):
            run(i)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(a.reps):
            run(i)
        e1.record()
        torch.cuda.synchronize()
        times[v].append(e0.elapsed_time(e1) / a.reps)
for v in variants:
    med = statistics.median(times[v])
    print(json.dumps({"config": "ralledata", "variant": v, "ms_median": med, "ms_min": min(times[v]),
                      "GBps": algo / med / 1e6, "frac_8TBps": algo / med / 1e6 / 8000}), flush=True)
