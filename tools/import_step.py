"""Driver for profiling bench.py's import secondary (k2himport TSV scan + prehash of an
8M-record file in HBM): builds bench.import_workload, warms up for ~150 ms, then runs
--calls calls of archive.import_scan_prehash_device.

    rocprofv3 ... -- python3 tools/import_step.py [--calls K]

With --mdbm: the same records in mdbm's print format (built on the device, records checked
against the generator and hashes against the ranges path), timed per call.

With --ab LIB: same-process A/B of the working tree's library against another build of it
(tools/build_ab.sh), interleaved rounds, each library's result checked against
tests/golden/import_digest.json first.
"""
import argparse
import ctypes
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import bench  # noqa: E402
from k2hash_amd import _native, archive  # noqa: E402


def _verify(out):
    recs, h1, h2 = out
    g = json.loads((ROOT / "tests" / "golden" / "import_digest.json").read_text())
    cols = {"key_off": recs[:, 0], "key_len": recs[:, 1], "val_off": recs[:, 2], "val_len": recs[:, 3],
            "h1": h1, "h2": h2}
    return g["records"] == recs.shape[0] and all(bench.digest_dev(v.contiguous(), 0) == g[k] for k, v in cols.items())


def mdbm_workload(dev):
    return bench.import_mdbm_workload(dev)


def verify_mdbm(out, data, exp):
    """Records equal the generator's; h1 / h2 equal the ranges path's C-string hashes of the
    same keys (k2h_amd_hash_ranges, CSTR: another product kernel, not the oracle)."""
    recs, h1, h2 = out
    if recs.shape != exp.shape or not torch.equal(recs, exp):
        return False
    g1, g2 = archive.hash_ranges(data, exp[:, 0].contiguous(), exp[:, 1].contiguous(), second=True, cstr=True)
    return bool(torch.equal(g1, h1) and torch.equal(g2, h2))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=10)
    ap.add_argument("--mdbm", action="store_true", help="time the mdbm scan (the same records in mdbm's print format)")
    ap.add_argument("--ab", default="", help="another build of libk2hash_amd.so to time against the tree's")
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--lib", default="", help="run (and profile) this build instead of the tree's")
    ap.add_argument("--no-parity", action="store_true", help="probe libraries (tools/probe_build.py): time without "
                    "the digest check (their results may be wrong by design)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    if a.lib:
        _native._batch = _native._bind(ctypes.CDLL(str(Path(a.lib).resolve())), _native.SIGNATURES.keys())
    if a.mdbm:  # one verified call, then the timed calls
        data, exp = mdbm_workload(dev)
        ok = verify_mdbm(archive.import_scan_prehash_device(data, "mdbm"), data, exp)
        print(json.dumps({"mdbm_bytes": data.numel(), "records": int(exp.shape[0]), "verify_ok": ok}), flush=True)
        if not ok and not a.no_parity:
            sys.exit(1)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.15:
            archive.import_scan_prehash_device(data, "mdbm")
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.rounds):
            t0 = time.perf_counter()
            for _ in range(a.calls):
                archive.import_scan_prehash_device(data, "mdbm")
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) / a.calls * 1e3)
        print(json.dumps({"mdbm_ms_per_call_median": statistics.median(ts), "min": min(ts), "all": ts}))
        return
    data = bench.import_workload(dev)
    if a.ab:
        libs = {"tree": _native.batch_lib()}
        for p in a.ab.split(","):
            libs[p] = _native._bind(ctypes.CDLL(str(Path(p).resolve())), _native.SIGNATURES.keys())
        for name, lib in libs.items():
            _native._batch = lib  # tool only: route archive's calls to this build
            ok = _verify(archive.import_scan_prehash_device(data))
            print(f"{name}: parity {'OK' if ok else 'MISMATCH'}", flush=True)
            if not ok and not (a.no_parity and name != "tree"):
                sys.exit(1)
        times = {k: [] for k in libs}
        for _ in range(a.rounds):
            for name, lib in libs.items():
                _native._batch = lib
                for _ in range(3):
                    archive.import_scan_prehash_device(data)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.calls):
                    archive.import_scan_prehash_device(data)
                torch.cuda.synchronize()
                times[name].append((time.perf_counter() - t0) / a.calls * 1e3)
        for name in libs:
            print(json.dumps({"lib": name, "ms_per_call_median": statistics.median(times[name]),
                              "ms_per_call_min": min(times[name]), "all": times[name]}), flush=True)
        return
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.15:
        archive.import_scan_prehash_device(data)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.calls):
        archive.import_scan_prehash_device(data)
    torch.cuda.synchronize()
    print(f"{(time.perf_counter() - t0) / a.calls * 1e3:.3f} ms per call")


if __name__ == "__main__":
    main()
