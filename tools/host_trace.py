#!/usr/bin/env python3
"""Run the fixed-key host path a few times (for rocprofv3 --sys-trace timelines of its
copies and kernels).  python tools/host_trace.py [--reps 3] [--n 16777216]"""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import k2hash_amd  # noqa: E402
from k2hash_amd import batch  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--reps", type=int, default=3)
p.add_argument("--n", type=int, default=1 << 24)
p.add_argument("--csr", action="store_true", help="CSR keys of 8-256 B instead of 32-byte keys")
a = p.parse_args()
dev = torch.device("cuda:0")
if a.csr:
    off = batch.synth_offsets(a.n, dev, 8, 256)
    data = batch.synth_bytes(int(off[-1].item()), dev).cpu().numpy()
    off = off.cpu().numpy().astype("uint64")
    run = lambda: k2hash_amd.hash_csr_host(data, off)  # noqa: E731
else:
    keys = batch.synth_bytes(a.n * 32, dev).cpu().numpy()
    run = lambda: k2hash_amd.hash_fixed_host(keys, 32)  # noqa: E731
for r in range(a.reps):
    t0 = time.perf_counter()
    run()
    print(f"rep {r}: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
