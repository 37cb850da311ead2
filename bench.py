#!/usr/bin/env python3
"""bench.py -- k2hash key-hash hot path on MI355X.

Headline (BASELINE.json metric, config 2): key hashes/s (device-resident) over
batched 32-byte keys -- one "step" = one batched launch hashing 16,777,216 keys
x 32 B (h1 only, as in the metric's 40 B/key algorithmic traffic), inputs already
resident in HBM.  Two input sets are rotated so the 256 MiB Infinity Cache cannot
hold the working set.  Multi-GPU (config 4 shape): each rank hashes its own
contiguous 16M-key shard (weak scaling, no collective inside the timed region);
with --gather the RCCL gather of the hashes to rank 0 is timed separately.

Prints ONE JSON line on rank 0 (contract in the task statement), with the
dominant kernel's roofline and a CPU baseline (the reference's own hash path,
oracle/_ref, timed on this host's cores; `port` when that build is absent).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config fixed32|csr|fixed4096]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    # name: (kind, keys per rank, key_len | (min,max), description)
    "fixed32": ("fixed", 1 << 24, 32, "16M x 32B fixed-length keys (BASELINE config 2)"),
    "csr": ("csr", 1 << 26, (8, 256), "64M mixed 8-256B keys, offsets+bytes CSR (BASELINE config 3)"),
    "fixed4096": ("fixed", 1 << 20, 4096, "1M x 4KiB keys (BASELINE config 5)"),
    # RALLEDATA blobs (hash + subhash + key + value) for a bulk direct set
    "ralledata": ("ralledata", 1 << 23, ((8, 64), (0, 256)),
                  "8M records (keys 8-64B, values 0-256B) -> RALLEDATA blobs with precomputed hashes"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--warm-ms", type=float, default=150.0,
                   help="keep warming up (untimed) until at least this much GPU time has passed: the "
                        "MI355X clock ramps over the first ~30 ms of back-to-back launches "
                        "(tools/clock_ramp.py, profiles/r01_clock_ramp.txt)")
    p.add_argument("--config", default="fixed32", choices=sorted(CONFIGS))
    p.add_argument("--second", action="store_true", help="also emit the second hash (h2)")
    p.add_argument("--gather", action="store_true", help="also time the RCCL gather of hashes (N>1)")
    p.add_argument("--index", action="store_true",
                   help="fused bucket-index epilogue (kindex + ckindex outputs, SURVEY 8f rank 1) with a "
                        "2^28-slot table: cur_mask 0x0FFFFFFF, collision_mask 0xF")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--variant", type=int, default=0, help="kernel variant (A/B knob, 0 = auto)")
    p.add_argument("--backend", default="nccl", help="torch.distributed backend for N>1 (nccl = RCCL)")
    return p.parse_args()


def cpu_baseline(keys_host, key_len, n):
    """Reference hash path on the host cores (rank 0, N=1 only).  Bounded sample:
    the first `n` keys of the benchmark workload, one pass single-threaded and one
    pass on `threads` threads."""
    import ctypes

    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle  # test/baseline infrastructure only

    lib = oracle.cpubench()
    so = str(oracle.REF_SO) if oracle.REF_SO.exists() else ""
    kind = "reference" if so else "port"
    threads = int(os.environ.get("K2H_CPU_THREADS", "16"))
    ptr = ctypes.c_void_p(keys_host.ctypes.data)
    dig = ctypes.c_uint64()
    t1 = lib.cpu_bench_fixed(so.encode(), ptr, key_len, n, 1, 1, 0, ctypes.byref(dig))
    tN = lib.cpu_bench_fixed(so.encode(), ptr, key_len, n, threads, 1, 0, ctypes.byref(dig))
    # k2hbench `-type rw` hash path, 100k loops (BASELINE config 1)
    tb = lib.cpu_bench_k2hbench(so.encode(), 100000, 100000, 1, ctypes.byref(dig))
    if t1 <= 0 or tN <= 0:
        return None
    return {
        "value": n / tN, "unit": "key hashes/s", "cores": threads, "kind": kind,
        "sample": f"first {n} keys of the same {key_len}B workload, h1 only, one pass on {threads} threads "
                  f"(reference lib/k2hashfunc.cc k2h_hash via dlsym)",
        "single_thread": n / t1,
        "k2hbench_rw_100k": {"seconds": tb, "hash_calls": 1000000, "calls_per_s": 1e6 / tb if tb > 0 else None,
                              "threads": 1},
    }


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    import k2hash_amd
    from k2hash_amd import batch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            print("for --gpus N > 1 launch with torch.distributed.run (one process per GPU)", file=sys.stderr)
            sys.exit(2)
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(ndev, 1))  # one process per GPU; wraps only in rehearsals
    torch.cuda.set_device(dev)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)
    batch.set_variant(args.variant)

    kind, n, shape, desc = CONFIGS[args.config]
    # --- synthetic input (global key range of this rank), two rotating sets ------------
    sets = []
    algo_bytes = 0
    for s in range(2):
        first = (s * world + rank) * n
        if kind == "fixed":
            keys = batch.synth_bytes(n * shape, dev, byte_off=first * shape)
            sets.append((keys, None))
            algo_bytes = n * shape + 8 * n
        elif kind == "ralledata":
            (klo, khi), (vlo, vhi) = shape
            ko = batch.synth_offsets(n, dev, klo, khi, first_key=first)
            vo = batch.synth_offsets(n, dev, vlo, vhi, seed=batch.SEED_LENS + 7, first_key=first)
            kb, vb = int(ko[-1].item()), int(vo[-1].item())
            kd = batch.synth_bytes(kb, dev, byte_off=s * (1 << 36) + rank * (1 << 34))
            vd = batch.synth_bytes(vb, dev, byte_off=s * (1 << 36) + rank * (1 << 34) + (1 << 33))
            blob = torch.empty(80 * n + kb + vb, dtype=torch.uint8, device=dev)
            boff = torch.empty(n + 1, dtype=torch.int64, device=dev)
            sets.append(((kd, ko, vd, vo), (blob, boff)))
            # minimal traffic: key + value bytes and their offsets in, blobs + blob offsets out
            algo_bytes = max(algo_bytes, (kb + vb + 16 * (n + 1)) + (80 * n + kb + vb + 8 * (n + 1)))
        else:
            off = batch.synth_offsets(n, dev, shape[0], shape[1], first_key=first)
            data = batch.synth_bytes(int(off[-1].item()), dev, byte_off=s * (1 << 36) + rank * (1 << 34))
            sets.append((data, off))
            algo_bytes = max(algo_bytes, int(off[-1].item()) + 8 * n + 8 * (n + 1))
    if args.second:
        algo_bytes += 8 * n
    if args.index:
        algo_bytes += 16 * n  # kindex + ckindex writes
    outs = [(torch.empty(n, dtype=torch.int64, device=dev),
             torch.empty(n, dtype=torch.int64, device=dev) if args.second else None) for _ in range(2)]
    idx = [(torch.empty(n, dtype=torch.int64, device=dev), torch.empty(n, dtype=torch.int64, device=dev))
           for _ in range(2)] if args.index else None
    torch.cuda.synchronize()
    lib = k2hash_amd._native.batch_lib()
    CUR_MASK, CMASK = (1 << 28) - 1, 0xF

    def step(i):
        keys, off = sets[i & 1]
        if kind == "ralledata":
            from k2hash_amd import ralledata
            (kd, ko, vd, vo), (blob, boff) = keys, off
            ralledata.build_ralledata(kd, ko, vd, vo, out=blob, blob_off=boff, total=blob.numel())
            return
        if args.index:
            import ctypes
            h1, h2 = outs[i & 1]
            k, c = idx[i & 1]
            p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
            s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            if kind == "fixed":
                rc = lib.k2h_amd_hash_fixed_index(p(keys), shape, n, p(h1), p(h2), 0, CUR_MASK, CMASK, p(k), p(c), s)
            else:
                rc = lib.k2h_amd_hash_csr_index(p(keys), p(off), n, p(h1), p(h2), 0, CUR_MASK, CMASK, p(k), p(c), s)
            k2hash_amd._native.check(rc)
        elif kind == "fixed":
            k2hash_amd.hash_fixed(keys, shape, second=args.second, out=outs[i & 1])
        else:
            k2hash_amd.hash_csr(keys, off, second=args.second, out=outs[i & 1])

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    w0 = time.perf_counter()
    extra = 0
    while (time.perf_counter() - w0) * 1e3 < args.warm_ms:
        for i in range(20):
            step(i)
        extra += 20
        torch.cuda.synchronize()
    # One event pair around the K back-to-back launches on the stream they run on:
    # kernel time per launch = (end - start) / K (inter-kernel gaps included, ~1-2 us).
    e_start, e_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e_start.record()
    for i in range(args.steps):
        step(i)
    e_end.record()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_avg_s = e_start.elapsed_time(e_end) / args.steps / 1e3
    total_keys = n * world * args.steps
    value = total_keys / elapsed

    gather = None
    if args.gather and world > 1:
        from k2hash_amd.shard import gather_hashes
        h = outs[0][0]
        for _ in range(2):
            gather_hashes(h)
        torch.cuda.synchronize()
        dist.barrier()
        g0 = time.perf_counter()
        for _ in range(5):
            gather_hashes(h)
        torch.cuda.synchronize()
        dist.barrier()
        gather = {"ms_per_gather": (time.perf_counter() - g0) / 5 * 1e3,
                  "bytes_to_root": 8 * n * (world - 1)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and kind == "fixed":
        m = n if shape <= 64 else max(1, (512 << 20) // shape)
        host = sets[0][0][: m * shape].cpu().numpy()
        cpu = cpu_baseline(host, shape, m)

    if rank == 0:
        achieved = algo_bytes / kern_avg_s / 1e9
        traffic = None
        prof = ROOT / "profiles" / f"traffic_{args.config}{'_index' if args.index else ''}{'_h2' if args.second else ''}.json"
        if prof.exists():
            traffic = json.loads(prof.read_text()).get("hbm_bytes_per_launch")
        key_bytes = n * (shape if kind == "fixed" else (shape[0][0] + shape[0][1]) / 2 if kind == "ralledata"
                         else (shape[0] + shape[1]) / 2)
        line = {
            "metric": "key hashes/sec + GiB/s (device-resident), batched 32B keys, 1 MI355X"
            if args.config == "fixed32" and not (args.index or args.second)
            else f"RALLEDATA records/sec (device-resident), {desc}" if kind == "ralledata"
            else f"key hashes{' + bucket indices' if args.index else ''}/sec (device-resident), {desc}",
            "value": value,
            "unit": "records/s" if kind == "ralledata" else "key hashes/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_extra_for_clock_ramp": extra,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64 (u8 key bytes in)",
            "data": "synthetic (splitmix64 counter stream, generated on device; SURVEY.md 8d spec in DESIGN.md)",
            "config": {"workload": desc, "keys_per_gpu": n,
                       "key_len": shape if kind == "fixed" else list(shape),
                       "second_hash": bool(args.second), "bucket_index": bool(args.index),
                       "parallelism": f"shard{world}",
                       "variant": args.variant},
            "key_gib_per_s": value * (key_bytes / n) / 2**30,
            "kernel_ms": kern_avg_s * 1e3,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                         "algorithmic_bytes_per_launch": algo_bytes},
            "cpu_baseline": cpu,
        }
        if gather:
            line["gather"] = gather
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
