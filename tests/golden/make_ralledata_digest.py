#!/usr/bin/env python3
"""Writes tests/golden/ralledata_digest.json: digests of the RALLEDATA blobs and blob
offsets of bench.py's ralledata workload (8M records: keys 8-64 B from the byte stream at
offset 0, values 0-256 B from offset 2^33, lengths from SEED_LENS / SEED_LENS + 7), built
by the oracle's layout restatement (oracle/fnv_oracle.c, pinned by tests/golden/ralledata.json)
over the oracle hash (pinned by the reference's own lib/k2hashfunc.cc).

Blob bytes are digested as little-endian uint64 words, zero-padded to a multiple of 8.

  python tests/golden/make_ralledata_digest.py [--n 8388608]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "oracle"))
import oracle  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=1 << 23)
a = p.parse_args()
n = a.n
ko = oracle.gen_offsets(n, 8, 64, oracle.SEED_LENS)
vo = oracle.gen_offsets(n, 0, 256, oracle.SEED_LENS + 7)
kb, vb = int(ko[-1]), int(vo[-1])
kd = oracle.gen_bytes(kb, oracle.SEED_BYTES, 0)
vd = oracle.gen_bytes(vb, oracle.SEED_BYTES, 1 << 33)
total = 80 * n + kb + vb
out = np.zeros((total + 7) // 8 * 8, np.uint8)
boff = np.zeros(n + 1, np.uint64)
L = oracle.lib()
L.oracle_build_ralledata(oracle._ptr(kd), oracle._ptr(ko), oracle._ptr(vd), oracle._ptr(vo), None, None, None, None,
                         n, oracle._ptr(out), oracle._ptr(boff), 0)
res = {"generator": "tests/golden/make_ralledata_digest.py (oracle restatement, oracle/fnv_oracle.c)",
       "n": n, "key_len": [8, 64], "val_len": [0, 256], "bytes": total,
       "blob": [f"{x:016x}" for x in oracle.digest(out.view(np.uint64))],
       "blob_off": [f"{x:016x}" for x in oracle.digest(boff)]}
(Path(__file__).resolve().parent / "ralledata_digest.json").write_text(json.dumps(res, indent=1) + "\n")
print(json.dumps(res))
