#!/usr/bin/env python3
"""Writes tests/golden/import_digest.json: digests of the records and key hashes that
k2himport's own TSV loop (tests/k2himport.cc:81-86, libstdc++ getline, restated in
oracle/gen_import.cc) produces for bench.py's import workload, each key hashed by the
REFERENCE's lib/k2hashfunc.cc as K2HShm::Set(const char*) passes it (key + NUL).

The workload (bench.py secondary "import", built on the device there from the same
generators): 2^23 records "key TAB value NEWLINE", key lengths 8-64 and value lengths
0-200 from the synthetic length streams (seeds SEED_LENS + 11 / + 13), bytes from the
synthetic byte stream at byte offset 2^34 mapped to printable ASCII (32 + b % 95).

The mdbm form (--mdbm, tests/golden/import_mdbm_digest.json; bench.py secondary
"import_mdbm"): the same records in mdbm's print format (tests/k2himport.cc:95-117), the
five header lines first, key and value each on their own line.

  make -C oracle ref && python tests/golden/make_import_digest.py [--mdbm]
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


MDBM_HDR = b"format=print\ntype=btree\nmdbm_pagesize=4096\nmdbm_pagecount=1\nHEADER=END\n"


def build(n: int = N, mdbm: bool = False) -> np.ndarray:
    """The TSV file, or (mdbm) the same records in mdbm's print format: the five header
    lines, then per record a key line and a value line (the TAB becomes a newline)."""
    kl = np.diff(oracle.gen_offsets(n, *KEY_LENS, seed=SEED_LENS + 11)).astype(np.int64)
    vl = np.diff(oracle.gen_offsets(n, *VAL_LENS, seed=SEED_LENS + 13)).astype(np.int64)
    h = len(MDBM_HDR) if mdbm else 0
    off = np.concatenate([[0], np.cumsum(kl + vl + 2)]) + h
    data = oracle.gen_bytes(int(off[-1]), byte_off=BYTE_OFF)
    data = (data % 95 + 32).astype(np.uint8)
    if mdbm:
        data[:h] = np.frombuffer(MDBM_HDR, dtype=np.uint8)
    data[off[:-1] + kl] = 10 if mdbm else 9
    data[off[1:] - 1] = 10
    return data


def main():
    mdbm = "--mdbm" in sys.argv[1:]
    gen = ROOT / "oracle" / "_ref" / "gen_import"
    data = build(mdbm=mdbm)
    with tempfile.NamedTemporaryFile(suffix=".mdbm" if mdbm else ".tsv", delete=False) as t:
        t.write(data.tobytes())
    try:
        out = json.loads(subprocess.run([str(gen), "mdbm-digest" if mdbm else "tsv-digest", t.name], check=True,
                                        capture_output=True, text=True).stdout)
    finally:
        os.unlink(t.name)
    out.update({"generator": f"tests/golden/make_import_digest.py{' --mdbm' if mdbm else ''} (oracle/_ref/gen_import "
                             f"{'mdbm' if mdbm else 'tsv'}-digest: k2himport's getline loop + the reference hash)",
                "bytes": int(data.size), "key_lens": KEY_LENS, "val_lens": VAL_LENS,
                "seeds": {"key_lens": SEED_LENS + 11, "val_lens": SEED_LENS + 13, "bytes_offset": BYTE_OFF}})
    if mdbm:
        out["header"] = MDBM_HDR.decode()
    name = "import_mdbm_digest.json" if mdbm else "import_digest.json"
    (Path(__file__).resolve().parent / name).write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
