#!/usr/bin/env python3
"""Host-to-host (PCIe-inclusive) rate of the batch ABI's host-pointer forms:
k2h_amd_hash_fixed_host / k2h_amd_hash_csr_host, keys in pageable host memory, hashes
back in host memory (the north_star's "starts and ends in host memory" path).  Also
prints the raw pinned H2D / D2H copy rates on the same box as the ceiling.

  python tools/host_rate.py [--reps 5]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import k2hash_amd  # noqa: E402
import oracle  # noqa: E402  (checker only)

p = argparse.ArgumentParser()
p.add_argument("--reps", type=int, default=5)
a = p.parse_args()


def best(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts), sorted(ts)[len(ts) // 2]


out = {}
# raw copy ceilings (pinned host <-> device, 512 MiB)
dev = torch.device("cuda:0")
hp = torch.empty(512 << 20, dtype=torch.uint8).pin_memory()
d = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
t, _ = best(lambda: (d.copy_(hp, non_blocking=True), torch.cuda.synchronize()), a.reps)
out["h2d_pinned_GBps"] = (512 << 20) / t / 1e9
t, _ = best(lambda: (hp.copy_(d, non_blocking=True), torch.cuda.synchronize()), a.reps)
out["d2h_pinned_GBps"] = (512 << 20) / t / 1e9
del hp, d

# config 2 shape, host form
n = 1 << 24
keys = oracle.gen_bytes(32 * n)
r1, _ = oracle.hash_fixed(keys[: 32 * 4096], 32)
h1, _ = k2hash_amd.hash_fixed_host(keys, 32)
assert np.array_equal(h1[:4096], r1), "host fixed32 parity"
t, med = best(lambda: k2hash_amd.hash_fixed_host(keys, 32), a.reps)
out["fixed32_16M_host"] = {"keys_per_s": n / t, "median_keys_per_s": n / med, "key_GBps": 32 * n / t / 1e9,
                           "bytes_moved_GBps": 40 * n / t / 1e9}
del keys

# config 3 shape at 1/8 size (8M keys, ~1.1 GB), host form
n = 1 << 23
off = oracle.gen_offsets(n, 8, 256)
data = oracle.gen_bytes(int(off[-1]))
h1, _ = k2hash_amd.hash_csr_host(data, off)
c1, _ = oracle.hash_csr(data, off[:4097])
assert np.array_equal(h1[:4096], c1), "host csr parity"
t, med = best(lambda: k2hash_amd.hash_csr_host(data, off), a.reps)
out["csr_8M_host"] = {"keys_per_s": n / t, "median_keys_per_s": n / med, "key_GBps": int(off[-1]) / t / 1e9,
                      "bytes_moved_GBps": (int(off[-1]) + 16 * n) / t / 1e9}
print(json.dumps(out, indent=1))
