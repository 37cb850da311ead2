#!/usr/bin/env python3
"""Run one lab kernel variant a few times on a BASELINE config (for rocprofv3 --pmc passes).
  python tools/run_variant.py --config csr --variant 64 [--reps 5]"""
import argparse
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
os.environ.setdefault("K2H_AMD_BATCH_LIB", str(ROOT / "tools" / "lab" / "libk2hash_amd_lab.so"))

import torch  # noqa: E402

import k2hash_amd  # noqa: E402
from k2hash_amd import _native, batch  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--config", default="csr", choices=["csr", "fixed32", "fixed4096", "ralledata"])
p.add_argument("--variant", type=int, default=0)
p.add_argument("--reps", type=int, default=5)
a = p.parse_args()
dev = torch.device("cuda:0")
_native.lab_set_variant(a.variant)
if a.config == "ralledata":  # bench.py's ralledata workload
    from k2hash_amd import ralledata
    n = 1 << 23
    ko = batch.synth_offsets(n, dev, 8, 64)
    vo = batch.synth_offsets(n, dev, 0, 256, seed=batch.SEED_LENS + 7)
    kb, vb = int(ko[-1].item()), int(vo[-1].item())
    kd, vd = batch.synth_bytes(kb, dev), batch.synth_bytes(vb, dev, byte_off=1 << 33)
    blob = torch.empty(80 * n + kb + vb, dtype=torch.uint8, device=dev)
    boff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    run = lambda: ralledata.build_ralledata(kd, ko, vd, vo, out=blob, blob_off=boff, total=blob.numel())  # noqa: E731
elif a.config == "csr":
    off = batch.synth_offsets(1 << 26, dev, 8, 256)
    data = batch.synth_bytes(int(off[-1].item()), dev)
    run = lambda: k2hash_amd.hash_csr(data, off)  # noqa: E731
else:
    L, n = (32, 1 << 24) if a.config == "fixed32" else (4096, 1 << 20)
    keys = batch.synth_bytes(n * L, dev)
    run = lambda: k2hash_amd.hash_fixed(keys, L)  # noqa: E731
for _ in range(a.reps):
    run()
torch.cuda.synchronize()
print("done", a.config, a.variant)
