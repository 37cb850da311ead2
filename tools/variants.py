#!/usr/bin/env python3
"""A/B timing of kernel variants in ONE process, interleaved rounds (rule: perf deltas
come from interleaved rounds in one process).  Each variant's output is checked
against the golden digest before it is timed.

  python tools/variants.py [--config fixed32|csr|fixed4096] [--variants 4,5,6] [--rounds 5] [--reps 10]
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
p.add_argument("--config", default="fixed32")
p.add_argument("--variants", default="0")
p.add_argument("--rounds", type=int, default=5)
p.add_argument("--reps", type=int, default=10)
p.add_argument("--second", action="store_true")
p.add_argument("--noparity", default="", help="comma list of variants whose parity is not checked (timing probes)")
a = p.parse_args()

dev = torch.device("cuda:0")
dig = json.loads((ROOT / "tests/golden/digests.json").read_text())["configs"]
name = {"fixed32": "fixed32_16M", "csr": "csr_8_256_64M", "fixed4096": "fixed4096_1M", "fixed21": "fixed21_1M"}[a.config]
cfg = dig[name]
n = cfg["n"]
sets = []
for s in range(2):
    if cfg["kind"] == "fixed":
        sets.append((batch.synth_bytes(n * cfg["key_len"], dev), None))
        algo = n * cfg["key_len"] + 8 * n
    else:
        off = batch.synth_offsets(n, dev, cfg["min_len"], cfg["max_len"])
        sets.append((batch.synth_bytes(int(off[-1].item()), dev), off))
        algo = int(off[-1].item()) + 16 * n + 8
if a.second:
    algo += 8 * n
out = (torch.empty(n, dtype=torch.int64, device=dev), torch.empty(n, dtype=torch.int64, device=dev))


def run(i):
    keys, off = sets[i & 1]
    o = (out[0], out[1] if a.second else None)
    if off is None:
        k2hash_amd.hash_fixed(keys, cfg["key_len"], second=a.second, out=o)
    else:
        k2hash_amd.hash_csr(keys, off, second=a.second, out=o)


variants = [int(v) for v in a.variants.split(",")]
for v in variants:
    _native.lab_set_variant(v)
    run(0)
    torch.cuda.synchronize()
    d1 = oracle.digest(out[0].cpu().numpy().view(np.uint64))
    ok = [f"{x:016x}" for x in d1] == cfg["h1"]
    if a.second:
        ok = ok and [f"{x:016x}" for x in oracle.digest(out[1].cpu().numpy().view(np.uint64))] == cfg["h2"]
    print(f"variant {v}: parity {'OK' if ok else 'MISMATCH'}", flush=True)
    if not ok and str(v) not in a.noparity.split(","):
        sys.exit(1)

import time  # noqa: E402
_native.lab_set_variant(variants[0])
w0 = time.perf_counter()
while time.perf_counter() - w0 < 0.3:  # past the clock ramp (profiles/r01_clock_ramp.txt)
    for i in range(10):
        run(i)
    torch.cuda.synchronize()
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
    print(json.dumps({"config": a.config, "variant": v, "ms_median": med, "ms_min": min(times[v]),
                      "GBps": algo / med / 1e6, "frac_8TBps": algo / med / 1e6 / 8000,
                      "Gkeys_s": n / med / 1e6}), flush=True)
