#!/usr/bin/env python3
"""ORACLE -- TEST INFRASTRUCTURE ONLY.  Writes the k2himport fixture:

  tests/golden/import/*.tsv, *.mdbm   small inputs covering the getline edge cases of
                                      tests/k2himport.cc:74-117 (keys spanning newlines,
                                      empty keys / values, NUL bytes, CR LF, high bytes,
                                      text after the last TAB, bad and short mdbm headers)
                                      plus a seeded 3000-record TSV and seeded
                                      small-alphabet fuzz files (fuzz_*)
  tests/golden/import.json            for each input, what oracle/_ref/gen_import prints:
                                      the records k2himport's own loops produce (libstdc++
                                      getline) and every key hashed by the REFERENCE's
                                      lib/k2hashfunc.cc as K2HShm::Set(const char*) passes it

Run after `make -C oracle ref` (needs /root/reference):  python3 oracle/gen_import_fixture.py
"""
import json
import random
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
OUT = ROOT / "tests" / "golden" / "import"
GEN = ROOT / "oracle" / "_ref" / "gen_import"

HDR = b"format=print\ntype=btree\nmdbm_version=3\nflags=0\nHEADER=END\n"
INPUTS = {
    "basic.tsv": b"key1\tvalue1\nkey2\tvalue2\n",
    "edge.tsv": (b"abc\ndef\tkey spans a newline\n"   # getline(.., '\t') reads across '\n'
                 b"\tempty key\n"
                 b"empty value\t\n"
                 b"nul\0inkey\tv\n"                    # c_str() cuts at the NUL
                 b"k\tnul\0invalue\n"
                 b"crlf\tvalue\r\n"
                 b"\x80\xff\xc3\xa9high\tbytes\n"
                 b"two\ttabs\tin line\n"               # value runs to the newline
                 b"\n\n\tnewlines before key\n"
                 b"trailing text without a tab"),       # eof inside the key getline: dropped
    "eof_value.tsv": b"k1\tv1\nk2\tlast value without newline",
    "eof_tab.tsv": b"k1\tv1\nlastkey\t",                # empty value at EOF still a record
    "empty.tsv": b"",
    "notab.tsv": b"no tab at all\nsecond line\n",
    "good.mdbm": HDR + b"k1\nv1\nk\0nul\nv\n\nempty key\nlastkey\n",  # last key: empty value
    "odd.mdbm": HDR + b"k1\nv1\nonly key",
    "bad.mdbm": b"format=print\ntype=btree\nmdbm_version=3\nflags=0\nHEADER=ENDX\nk\nv\n",
    "short.mdbm": b"format=print\nHEADER=END\n",
}


def random_tsv(n=3000, seed=7):
    rng = random.Random(seed)
    lines = []
    for _ in range(n):
        klen = rng.randint(0, 60)
        key = bytes(rng.choice([b for b in range(256) if b != 9]) for _ in range(klen))
        vlen = rng.randint(0, 120)
        val = bytes(rng.choice([b for b in range(256) if b != 10]) for _ in range(vlen))
        lines.append(key + b"\t" + val + b"\n")
    return b"".join(lines)


def fuzz_inputs(seed=0x6B32):
    """Small-alphabet files (TAB, newline, NUL, high bytes frequent: keys across lines,
    values with TABs and NULs, every EOF shape) at sizes around the device scanner's
    64-byte thread span and 16 KiB block (k2hash_amd/csrc/k2h_import_dev.hip)."""
    rng = random.Random(seed)
    alphabet = b"ab\t\n\x00c\xff"
    weights = [30, 25, 12, 18, 5, 5, 5]
    out = {}
    for size in (1, 2, 3, 5, 8, 13, 21, 34, 55, 63, 64, 65, 127, 128, 129, 300, 1000, 4097, 16383, 16384, 16385):
        out[f"fuzz_{size:05d}.tsv"] = bytes(rng.choices(alphabet, weights, k=size))
    for size in (0, 1, 2, 3, 5, 8, 13, 64, 65, 300, 4097):
        out[f"fuzz_{size:05d}.mdbm"] = HDR + bytes(rng.choices(alphabet, weights, k=size))
    return out


def main():
    OUT.mkdir(parents=True, exist_ok=True)
    inputs = dict(INPUTS)
    inputs["random.tsv"] = random_tsv()
    inputs.update(fuzz_inputs())
    fixture = {"generator": "oracle/_ref/gen_import (tests/k2himport.cc loops, reference lib/k2hashfunc.cc)",
               "inputs": {}}
    for name, data in sorted(inputs.items()):
        (OUT / name).write_bytes(data)
        fmt = "mdbm" if name.endswith(".mdbm") else "tsv"
        res = json.loads(subprocess.run([str(GEN), fmt, str(OUT / name)], check=True, capture_output=True,
                                        text=True).stdout)
        fixture["inputs"][name] = res
    (ROOT / "tests" / "golden" / "import.json").write_text(json.dumps(fixture, indent=1) + "\n")
    print({k: len(v["records"]) for k, v in fixture["inputs"].items()})


if __name__ == "__main__":
    main()
