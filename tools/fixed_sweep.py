#!/usr/bin/env python3
"""Fixed-length key sweep: time the fixed-key kernels (variant 9 per-lane tail loop,
10 per-lane direct loads, 11/0 line ring) over key lengths, interleaved in one process,
to pick the routing crossover in launch_fixed.  Parity of every variant/length is
checked against the oracle on the first 4096 keys.

  python tools/fixed_sweep.py [--lens 8,21,48,64,100,128,256,1024] [--variants 9,10,11]
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import os  # noqa: E402
os.environ.setdefault("K2H_AMD_BATCH_LIB", str(Path(__file__).resolve().parents[1] / "tools" / "lab" / "libk2hash_amd_lab.so"))
import k2hash_amd  # noqa: E402
from k2hash_amd import _native  # noqa: E402
from k2hash_amd import batch  # noqa: E402
import oracle  # noqa: E402  (checker only)

p = argparse.ArgumentParser()
p.add_argument("--lens", default="8,16,21,24,48,64,100,128,256,1024")
p.add_argument("--variants", default="9,10,11")
p.add_argument("--bytes", type=int, default=512 << 20, help="key bytes per launch")
p.add_argument("--rounds", type=int, default=3)
p.add_argument("--reps", type=int, default=10)
a = p.parse_args()
dev = torch.device("cuda:0")
variants = [int(v) for v in a.variants.split(",")]
for L in [int(x) for x in a.lens.split(",")]:
    n = a.bytes // L
    keys = batch.synth_bytes(n * L, dev)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    ref = oracle.hash_fixed(keys[: 4096 * L].cpu().numpy(), L)[0]
    for v in variants:
        _native.lab_set_variant(v)
        k2hash_amd.hash_fixed(keys, L, out=(out, None))
        torch.cuda.synchronize()
        if not np.array_equal(out[:4096].cpu().numpy().view(np.uint64), ref):
            print(f"L={L} variant {v}: MISMATCH", flush=True)
            sys.exit(1)
    times = {v: [] for v in variants}
    for r in range(a.rounds):
        for v in variants:
            _native.lab_set_variant(v)
            for i in range(2):
                k2hash_amd.hash_fixed(keys, L, out=(out, None))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(a.reps):
                k2hash_amd.hash_fixed(keys, L, out=(out, None))
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.reps)
    row = {"L": L, "n": n}
    for v in variants:
        med = statistics.median(times[v])
        row[f"v{v}_ms"] = round(med, 4)
        row[f"v{v}_frac"] = round((n * L + 8 * n) / med / 1e6 / 8000, 3)
    print(json.dumps(row), flush=True)
    del keys, out
    _native.lab_set_variant(0)
