#!/usr/bin/env python3
"""Does the fixed32 launch time depend on how long the GPU has been busy (clock ramp)?
Runs N back-to-back launches with per-launch event pairs and prints the median
duration of each block of 50 launches, then a long-warmup K-launch event pair."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import os  # noqa: E402
os.environ.setdefault("K2H_AMD_BATCH_LIB", str(Path(__file__).resolve().parents[1] / "tools" / "lab" / "libk2hash_amd_lab.so"))
import k2hash_amd  # noqa: E402
from k2hash_amd import _native  # noqa: E402
from k2hash_amd import batch  # noqa: E402

dev = torch.device("cuda:0")
n = 1 << 24
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
variant = int(sys.argv[2]) if len(sys.argv) > 2 else 0
_native.lab_set_variant(variant)
sets = [batch.synth_bytes(32 * n, dev, byte_off=s * 32 * n) for s in range(2)]
outs = [torch.empty(n, dtype=torch.int64, device=dev) for _ in range(2)]


def step(i):
    k2hash_amd.hash_fixed(sets[i & 1], 32, out=(outs[i & 1], None))


torch.cuda.synchronize()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(N)]
for i in range(N):
    ev[i][0].record()
    step(i)
    ev[i][1].record()
torch.cuda.synchronize()
d = [x.elapsed_time(y) * 1e3 for x, y in ev]
for b in range(0, N, 50):
    blk = sorted(d[b:b + 50])
    print(f"launches {b:5d}-{b + len(blk) - 1:5d}: median {blk[len(blk) // 2]:8.2f} us  min {blk[0]:8.2f}")
for K in (20, 100, 400):
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(K):
        step(i)
    e.record()
    torch.cuda.synchronize()
    print(f"after warm: pair around {K} launches: {a.elapsed_time(e) / K * 1e3:8.2f} us/launch")
