#!/usr/bin/env python3
"""Build a PROBE copy of the batch library: the working tree's k2hash_amd/csrc copied to a
scratch directory, string replacements applied (each must match exactly once), built, and
the library copied to k2hash_amd/lib/probe/<name>.so.  Probes are timing experiments that
may break results (e.g. "no miss hashing"); they never touch the product sources.

  python tools/probe_build.py NAME FILE 'OLD' 'NEW' [FILE 'OLD' 'NEW' ...]
"""
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def main():
    name, edits = sys.argv[1], sys.argv[2:]
    assert len(edits) % 3 == 0
    tmp = Path(tempfile.mkdtemp(prefix="k2h_probe_"))
    shutil.copytree(ROOT / "k2hash_amd" / "csrc", tmp / "k2hash_amd" / "csrc")
    shutil.copytree(ROOT / "include", tmp / "include")
    for i in range(0, len(edits), 3):
        f = tmp / "k2hash_amd" / "csrc" / edits[i]
        s = f.read_text()
        assert s.count(edits[i + 1]) == 1, (edits[i], edits[i + 1][:60], s.count(edits[i + 1]))
        f.write_text(s.replace(edits[i + 1], edits[i + 2]))
    subprocess.run(["make", "-C", str(tmp / "k2hash_amd" / "csrc"), "-j8"], check=True, stdout=subprocess.DEVNULL)
    out = ROOT / "k2hash_amd" / "lib" / "probe"
    out.mkdir(parents=True, exist_ok=True)
    shutil.copy(tmp / "k2hash_amd" / "lib" / "libk2hash_amd.so", out / f"{name}.so")
    shutil.rmtree(tmp)
    print(out / f"{name}.so")


if __name__ == "__main__":
    main()
