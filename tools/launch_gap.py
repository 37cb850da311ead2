#!/usr/bin/env python3
"""Where does the time between back-to-back fixed32 launches go?  Compares, on the same
buffers: one event pair around K launches; per-launch event pairs; host enqueue time;
and K launches captured in a HIP graph (torch.cuda.CUDAGraph) and replayed."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import k2hash_amd  # noqa: E402
from k2hash_amd import batch  # noqa: E402

dev = torch.device("cuda:0")
n = 1 << 24
K = 20
sets = [batch.synth_bytes(32 * n, dev, byte_off=s * 32 * n) for s in range(2)]
outs = [torch.empty(n, dtype=torch.int64, device=dev) for _ in range(2)]


def step(i, stream=None):
    k2hash_amd.hash_fixed(sets[i & 1], 32, out=(outs[i & 1], None), stream=stream)


for i in range(5):
    step(i)
torch.cuda.synchronize()
for rep in range(3):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record()
    for i in range(K):
        step(i)
    t1 = time.perf_counter()
    b.record()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"pair: {a.elapsed_time(b) / K * 1e3:8.2f} us/launch  host enqueue {(t1 - t0) / K * 1e6:7.2f} us/launch  "
          f"wall {(t2 - t0) / K * 1e6:8.2f} us/launch")
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
for i in range(K):
    ev[i][0].record()
    step(i)
    ev[i][1].record()
torch.cuda.synchronize()
per = sorted(x.elapsed_time(y) * 1e3 for x, y in ev)
print(f"per-launch pairs: median {per[K // 2]:8.2f} us  min {per[0]:8.2f}  max {per[-1]:8.2f}")
# HIP graph
s = torch.cuda.Stream()
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(s):
    step(0, stream=s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        for i in range(K):
            step(i, stream=s)
torch.cuda.synchronize()
for rep in range(3):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    torch.cuda.synchronize()
    print(f"graph: {a.elapsed_time(b) / K * 1e3:8.2f} us/launch")
