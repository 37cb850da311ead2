#!/usr/bin/env python3
"""Writes tests/golden/import_digest.json: digests of the records and key hashes that
k2himport's own TSV loop (tests/k2himport.cc:81-86, libstdc++ getline, restated in
oracle/gen_import.cc) produces for bench.py's import workload, each key hashed by the
REFERENCE's lib/k2hashfunc.cc as K2HShm::Set(const char*) passes it (key + NUL).

The workload (bench.py secondary "import", built on the device there from the same
generators): 2^23 records "key TAB value NEWLINE", key lengths 8-64 and value lengths
0-200 from the synthetic length streams (seeds SEED_LENS + 11 / + 13), bytes from the
synthetic byte stream at byte offset 2^34 mapped to printable ASCII (32 + b % 95).

  make -C oracle ref && python tests/golden/make_import_digest.py
"""
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "oracle"))
import oracle  # noqa: E402

N = 1 << 23
SEED_LENS = 0x6B32686173680002
KEY_LENS, VAL_LENS = (8, 64), (0, 200)
BYTE_OFF = 1 << 34


def build(n: int = N) -> np.ndarray:
    kl = np.diff(oracle.gen_offsets(n, *KEY_LENS, seed=SEED_LENS + 11)).astype(np.int64)
    vl = np.diff(oracle.gen_offsets(n, *VAL_LENS, seed=SEED_LENS + 13)).astype(np.int64)
    off = np.concatenate([[0], np.cumsum(kl + vl + 2)])
    data = oracle.gen_bytes(int(off[-1]), byte_off=BYTE_OFF)
    data = (data % 95 + 32).astype(np.uint8)
    data[off[:-1] + kl] = 9
    data[off[1:] - 1] = 10
    return data


def main():
    gen = ROOT / "oracle" / "_ref" / "gen_import"
    data = build()
    with tempfile.NamedTemporaryFile(suffix=".tsv", delete=False) as t:
        t.write(data.tobytes())
    try:
        out = json.loads(subprocess.run([str(gen), "tsv-digest", t.name], check=True, capture_output=True,
                                        text=True).stdout)
    finally:
        os.unlink(t.name)
    out.update({"generator": "tests/golden/make_import_digest.py (oracle/_ref/gen_import tsv-digest: "
                             "k2himport's getline loop + the reference hash)",
                "bytes": int(data.size), "key_lens": KEY_LENS, "val_lens": VAL_LENS,
                "seeds": {"key_lens": SEED_LENS + 11, "val_lens": SEED_LENS + 13, "bytes_offset": BYTE_OFF}})
    (Path(__file__).resolve().parent / "import_digest.json").write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
