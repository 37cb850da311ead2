#!/usr/bin/env python3
"""Writes tests/golden/index_digest.json: digests of the bucket positions (kindex, ckindex)
of BASELINE config 2 (16M x 32 B keys, the bench's byte stream) for bench.py's fused-index
secondary result (cur_mask = 2^28 - 1, collision_mask = 0xF).  h1 from the oracle hash,
positions from the oracle's restatement of GetKIndexPos / GetCKIndex (oracle/fnv_oracle.c,
lib/k2hshm.cc:78-90, 810-833, 1093; pinned by the dsave fixture and the key_index_area
table, tests/test_bucket_index.py).

  python tests/golden/make_index_digest.py
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "oracle"))
import oracle  # noqa: E402

N, L = 1 << 24, 32
CUR_MASK, CMASK = (1 << 28) - 1, 0xF
keys = oracle.gen_bytes(N * L)
h1, _ = oracle.hash_fixed(keys, L)
k, c = oracle.bucket_index(h1, CUR_MASK, CMASK)
res = {"generator": "tests/golden/make_index_digest.py (oracle hash + oracle bucket index)",
       "n": N, "key_len": L, "cur_mask": CUR_MASK, "collision_mask": CMASK,
       "h1": [f"{x:016x}" for x in oracle.digest(h1)],
       "kindex": [f"{x:016x}" for x in oracle.digest(k)],
       "ckindex": [f"{x:016x}" for x in oracle.digest(c)]}
(Path(__file__).resolve().parent / "index_digest.json").write_text(json.dumps(res, indent=1) + "\n")
print(json.dumps(res))
