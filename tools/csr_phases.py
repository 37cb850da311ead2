#!/usr/bin/env python3
"""Where does a CSR tile's time go?  Runs the staged CSR kernel in its profiling mode
(variant 15: h2 receives, per 512-key tile, 100 MHz wall-clock stamps at the phase
boundaries and each wave's finish) over BASELINE config 3 and summarises:
  load   = offsets -> LDS (+ first barrier)
  sort   = histogram / scan / scatter (+ DMA issue)
  wait   = DMA drain + barrier
  hash   = chunk walk of the slowest wave; imbalance = slowest - fastest wave
plus per-CU residency (how many tiles overlap on a CU on average), the kernel's span
and the tail after the last tile starts.

  python tools/csr_phases.py [--n 67108864]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import os  # noqa: E402
os.environ.setdefault("K2H_AMD_BATCH_LIB", str(Path(__file__).resolve().parents[1] / "tools" / "lab" / "libk2hash_amd_lab.so"))
import k2hash_amd  # noqa: E402
from k2hash_amd import _native  # noqa: E402
from k2hash_amd import batch  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=1 << 26)
p.add_argument("--min-len", type=int, default=8)
p.add_argument("--max-len", type=int, default=256)
a = p.parse_args()
dev = torch.device("cuda:0")
off = batch.synth_offsets(a.n, dev, a.min_len, a.max_len)
data = batch.synth_bytes(int(off[-1].item()), dev)
tiles = (a.n + 511) // 512
h1 = torch.empty(a.n, dtype=torch.int64, device=dev)
stamps = torch.zeros(16 * tiles + 16, dtype=torch.int64, device=dev)
# reference timing with the default kernel
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(3):
    k2hash_amd.hash_csr(data, off, out=(h1, None))
e0.record()
for _ in range(5):
    k2hash_amd.hash_csr(data, off, out=(h1, None))
e1.record()
torch.cuda.synchronize()
ms_default = e0.elapsed_time(e1) / 5
ref = h1.clone()
_native.lab_set_variant(15)
for _ in range(3):
    k2hash_amd.hash_csr(data, off, out=(h1, stamps))
e0.record()
k2hash_amd.hash_csr(data, off, out=(h1, stamps))
e1.record()
torch.cuda.synchronize()
ms_prof = e0.elapsed_time(e1)
_native.lab_set_variant(0)
assert torch.equal(h1, ref), "profiling mode changed the hashes"
s = stamps[: 16 * tiles].view(tiles, 16).cpu().numpy()
t = s[:, :8].astype(np.float64) * 10.0  # ns (100 MHz)
t0 = t[:, 0].min()
t -= t0
sub = s[:, 10:13].astype(np.float64) * 10.0 - t0
dma_issue = sub[:, 0] - t[:, 1]
hist = sub[:, 1] - sub[:, 0]
scan = sub[:, 2] - sub[:, 1]
scatter = t[:, 2] - sub[:, 2]
hw = s[:, 8].astype(np.uint64)
staged = s[:, 9]
wave_end = t[:, 4:8]
load = t[:, 1] - t[:, 0]
sort = t[:, 2] - t[:, 1]
wait = t[:, 3] - t[:, 2]
hash_ = wave_end.max(1) - t[:, 3]
imb = wave_end.max(1) - wave_end.min(1)
life = wave_end.max(1) - t[:, 0]
hwid = hw & 0xFFFFFFFF
xcc = (hw >> 32) & 0xF
cu = (hwid >> 8) & 0xF
sh = (hwid >> 12) & 0x1
se = (hwid >> 13) & 0x7
cu_key = (xcc << 8) | (se << 5) | (sh << 4) | cu
ucu = np.unique(cu_key)
span = wave_end.max()
busy = np.zeros(len(ucu))
for i, c in enumerate(ucu):
    busy[i] = life[cu_key == c].sum()
res = {
    "n": a.n, "tiles": tiles, "ms_default": ms_default, "ms_prof_launch": ms_prof,
    "span_us_from_first_stamp": span / 1e3, "cus_seen": int(len(ucu)), "staged_frac": float(staged.mean()),
    "mean_us": {"load": load.mean() / 1e3, "sort": sort.mean() / 1e3,
                "sort.dma_issue": dma_issue.mean() / 1e3, "sort.histogram": hist.mean() / 1e3,
                "sort.scan": scan.mean() / 1e3, "sort.scatter": scatter.mean() / 1e3, "dma_wait": wait.mean() / 1e3,
                "hash_slowest_wave": hash_.mean() / 1e3, "wave_imbalance": imb.mean() / 1e3,
                "tile_life": life.mean() / 1e3},
    "p99_us": {"tile_life": float(np.percentile(life, 99)) / 1e3, "hash": float(np.percentile(hash_, 99)) / 1e3},
    "tiles_resident_per_cu_avg": float(busy.mean() / span),
    "cu_busy_spread": {"min": float(busy.min() / span), "max": float(busy.max() / span)},
    "last_tile_start_us": float(t[:, 0].max() / 1e3),
    "tail_us": float((span - t[:, 0].max()) / 1e3),
}
print(json.dumps(res, indent=1))
