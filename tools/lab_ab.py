#!/usr/bin/env python3
"""Round-3 lab A/B: interleaved timing of tools/lab/libk2hash_lab.so variants against the
product launch, each result digest-checked against the reference first.

  python tools/lab_ab.py lines --variants 0:0 1:8 1:10 [--reps 5 --launches 20]
      config 5 (1M x 4 KiB): variant:waves_per_cu
  python tools/lab_ab.py csr --variants 0 1 2
      config 3 (64M CSR keys)
  python tools/lab_ab.py ralle --variants 0 1
      bench's RALLEDATA workload (8M records)

Prints one JSON object (per-variant median / min launch time in microseconds)."""
from __future__ import annotations

import argparse
import ctypes
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402  (digest helpers)

_p, _u64 = ctypes.c_void_p, ctypes.c_uint64


def lab_lib():
    lib = ctypes.CDLL(str(ROOT / "tools" / "lab" / "libk2hash_lab.so"))
    if hasattr(lib, "k2h_lab_lines"):
        lib.k2h_lab_lines.restype = ctypes.c_int
        lib.k2h_lab_lines.argtypes = [ctypes.c_int, _p, _u64, _u64, _p, _p, ctypes.c_int, _p]
    if hasattr(lib, "k2h_lab_csr"):
        lib.k2h_lab_csr.restype = ctypes.c_int
        lib.k2h_lab_csr.argtypes = [ctypes.c_int, _p, _p, _u64, _p, _p, _p]
    if hasattr(lib, "k2h_lab_csr_rs"):
        lib.k2h_lab_csr_rs.restype = ctypes.c_int
        lib.k2h_lab_csr_rs.argtypes = [ctypes.c_int, _p, _p, _u64, _p, _p, _p]
        lib.k2h_lab_csr_rs2.restype = ctypes.c_int
        lib.k2h_lab_csr_rs2.argtypes = [ctypes.c_int, _p, _p, _u64, _p, _p, _p]
        lib.k2h_lab_csr_rs4.restype = ctypes.c_int
        lib.k2h_lab_csr_rs4.argtypes = [ctypes.c_int, _p, _p, _u64, _p, _p, _p]
        lib.k2h_lab_csr_lean.restype = ctypes.c_int
        lib.k2h_lab_csr_lean.argtypes = [ctypes.c_int, _p, _p, _u64, _p, _p, _p]
        lib.k2h_lab_csr_lean4.restype = ctypes.c_int
        lib.k2h_lab_csr_lean4.argtypes = [ctypes.c_int, _p, _p, _u64, _p, _p, _p]
        lib.k2h_lab_simd_probe.restype = ctypes.c_int
        lib.k2h_lab_simd_probe.argtypes = [_p, ctypes.c_uint, _p]
    if hasattr(lib, "k2h_lab_ralle"):
        lib.k2h_lab_ralle.restype = ctypes.c_int
        lib.k2h_lab_ralle.argtypes = [ctypes.c_int, _p, _p, _p, _p, _u64, _p, _p, _p]
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", choices=["lines", "csr", "ralle"])
    ap.add_argument("--variants", nargs="+", required=True)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--warm-ms", type=float, default=200.0)
    ap.add_argument("--simd-probe", action="store_true")
    ap.add_argument("--rs-stats", action="store_true")
    ap.add_argument("--rs-steps", action="store_true")
    ap.add_argument("--rs2-stats", action="store_true")
    args = ap.parse_args()

    import torch

    from k2hash_amd import batch

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    lib = lab_lib()
    stream = torch.cuda.current_stream()
    sh = ctypes.c_void_p(stream.cuda_stream)
    gold = bench._golden()
    if args.config == "lines":
        n, L = 1 << 20, 4096
        keys = batch.synth_bytes(n * L, dev)
        h1 = torch.empty(n, dtype=torch.int64, device=dev)
        g = gold["fixed4096_1M"]
        chunks = g.get("chunks") or [dict(first=0, count=g["n"], h1=g["h1"])]

        def launch(v):
            var, wpc = (int(x) for x in v.split(":"))
            rc = lib.k2h_lab_lines(var, ctypes.c_void_p(keys.data_ptr()), L, n, ctypes.c_void_p(h1.data_ptr()),
                                   None, wpc, sh)
            assert rc == 0, rc
    elif args.config == "ralle":
        _, n, ((klo, khi), (vlo, vhi)), _ = bench.CONFIGS["ralledata"]
        ko = batch.synth_offsets(n, dev, klo, khi)
        vo = batch.synth_offsets(n, dev, vlo, vhi, seed=batch.SEED_LENS + 7)
        kb, vb = int(ko[-1].item()), int(vo[-1].item())
        kd = batch.synth_bytes(kb, dev)
        vd = batch.synth_bytes(vb, dev, byte_off=1 << 33)
        total = 80 * n + kb + vb
        blob = torch.zeros((total + 7) // 8 * 8, dtype=torch.uint8, device=dev)
        boff = torch.empty(n + 1, dtype=torch.int64, device=dev)
        g = json.loads((ROOT / "tests" / "golden" / "ralledata_digest.json").read_text())
        h1 = None

        def launch(v):
            rc = lib.k2h_lab_ralle(int(v), ctypes.c_void_p(kd.data_ptr()), ctypes.c_void_p(ko.data_ptr()),
                                   ctypes.c_void_p(vd.data_ptr()), ctypes.c_void_p(vo.data_ptr()), n,
                                   ctypes.c_void_p(blob.data_ptr()), ctypes.c_void_p(boff.data_ptr()), sh)
            assert rc == 0, rc

        def verify():
            ok = g["n"] == n and g["bytes"] == total and bench.digest_dev(blob.view(torch.int64), 0) == g["blob"] \
                and bench.digest_dev(boff, 0) == g["blob_off"]
            return {"ok": ok}
    else:
        n = 1 << 26
        off = batch.synth_offsets(n, dev, 8, 256)
        data = batch.synth_bytes(int(off[-1].item()), dev)
        h1 = torch.empty(n, dtype=torch.int64, device=dev)
        chunks = gold["csr_8_256_64M"]["chunks"]

        def launch(v):
            # 20-27: lab_csr_rs.inc, 30-33: lab_csr_rs2.inc, 40-42: lab_csr_rs4.inc, 50-54: lab_csr_lean.inc
            fn = (lib.k2h_lab_csr_lean4 if int(v) >= 53 else lib.k2h_lab_csr_lean if int(v) >= 50 else lib.k2h_lab_csr_rs4 if int(v) >= 40 else lib.k2h_lab_csr_rs2 if int(v) >= 30 else
                  lib.k2h_lab_csr_rs if int(v) >= 20 else lib.k2h_lab_csr)
            rc = fn(int(v), ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(off.data_ptr()), n,
                    ctypes.c_void_p(h1.data_ptr()), None, sh)
            assert rc == 0, rc

        if args.simd_probe:  # SIMD (HW_ID bits 5:4) of each wave of the first 4 blocks of 512 threads
            out = torch.zeros(64, dtype=torch.int32, device=dev)
            assert lib.k2h_lab_simd_probe(ctypes.c_void_p(out.data_ptr()), 4, sh) == 0
            torch.cuda.synchronize()
            hw = [int(x) & 0xFFFFFFFF for x in out[:32].cpu()]
            print(json.dumps({"hw_id": [hex(h) for h in hw],
                              "simd_of_wave": [[(h >> 4) & 3 for h in hw[8 * b:8 * b + 8]] for b in range(4)]}))
        if args.rs_steps:  # executed walk steps per hash wave and tile (pairs of sorted ranks i, 511-i)
            import numpy as np
            o = off.cpu().numpy()
            k = (np.diff(o) + 15) // 16
            nt = n // 512
            k = np.sort(np.minimum(k[:nt * 512], 63).reshape(nt, 512), axis=1)
            A, B = k[:, :256].reshape(nt, 4, 64), k[:, ::-1][:, :256].reshape(nt, 4, 64)
            print(json.dumps({"rs_steps_per_wave_tile": {
                "pair_max": float((A + B).max(-1).mean()), "phase_max": float((A.max(-1) + B.max(-1)).mean()),
                "ideal": float((A + B).mean()), "tiles_per_cu": nt / 256}}))
        if args.rs2_stats:  # variant 33: rs2 with per-hash-wave phase clocks (8 hash waves)
            st = torch.zeros(256 * 8 * 8, dtype=torch.int64, device=dev)
            for _ in range(3):
                rc = lib.k2h_lab_csr_rs2(33, ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(off.data_ptr()), n,
                                         ctypes.c_void_p(h1.data_ptr()), ctypes.c_void_p(st.data_ptr()), sh)
                assert rc == 0, rc
            torch.cuda.synchronize()
            a = st.view(256, 8, 8)[:, :, :5].cpu().double()
            us = a[:, :, :4].mean(0) * 0.01  # per hash wave index, ticks (100 MHz) -> us
            print(json.dumps({"rs2_stats_us_by_wave": {"ready_wait": us[:, 0].tolist(), "prologue": us[:, 1].tolist(),
                              "walk": us[:, 2].tolist(), "epilogue_done": us[:, 3].tolist()},
                              "steps_by_wave": a[:, :, 4].mean(0).tolist(),
                              "verify": bench.verify_chunks(h1, 0, chunks)}))
        if args.rs_stats:  # variant 23: the role-split kernel with per-hash-wave phase clocks
            st = torch.zeros(256 * 4 * 8, dtype=torch.int64, device=dev)
            for _ in range(3):
                rc = lib.k2h_lab_csr_rs(23, ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(off.data_ptr()), n,
                                        ctypes.c_void_p(h1.data_ptr()), ctypes.c_void_p(st.data_ptr()), sh)
                assert rc == 0, rc
            torch.cuda.synchronize()
            a = st.view(-1, 8)[:, :5].cpu().double()
            us = a[:, :4].mean(0) * 0.01  # memrealtime ticks (100 MHz) -> us
            steps = a[:, 4].mean().item()
            print(json.dumps({"rs_stats_us_per_hash_wave": {"prologue": us[0].item(), "walk": us[1].item(),
                              "epilogue": us[2].item(), "barrier": us[3].item()},
                              "steps_per_hash_wave": steps, "walk_ns_per_step": us[1].item() * 1e3 / steps,
                              "verify": bench.verify_chunks(h1, 0, chunks)}))

    res = {}
    for v in args.variants:  # parity first
        if args.config == "ralle":
            blob.zero_()
            boff.zero_()
            launch(v)
            torch.cuda.synchronize()
            res[v] = {"verify": verify()}
            continue
        h1.zero_()
        launch(v)
        torch.cuda.synchronize()
        res[v] = {"verify": bench.verify_chunks(h1, 0, chunks)}
    import time
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < args.warm_ms:
        for v in args.variants:
            launch(v)
        torch.cuda.synchronize()
    times = {v: [] for v in args.variants}
    for _ in range(args.reps):
        for v in args.variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.launches):
                launch(v)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) * 1e3 / args.launches)
    for v in args.variants:
        res[v].update({"median_us": statistics.median(times[v]), "min_us": min(times[v]), "all_us": times[v]})
    print(json.dumps({"config": args.config, "n": n, "results": res}))


if __name__ == "__main__":
    main()
