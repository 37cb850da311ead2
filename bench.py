#!/usr/bin/env python3
"""bench.py -- k2hash key-hash hot path on MI355X.

Headline (BASELINE.json metric, config 2): key hashes/s (device-resident) over batched
32-byte keys -- one "step" = one batched launch hashing 16,777,216 keys x 32 B (h1 only,
40 B/key of algorithmic traffic), inputs already resident in HBM; two input sets are
rotated so the 256 MiB Infinity Cache cannot hold the working set.

--gpus N > 1 (config 4: 2^30 x 32 B keys over N GPUs, strong scaling): one process per
GPU.  Launched by torch.distributed.run (RANK / WORLD_SIZE in the environment) or, when
those are absent, by this script itself: it starts N fresh child processes before
touching any GPU and relays rank 0's line.  Each rank hashes its contiguous shard of the
2^30 keys (no data-path collective: keys are independent, lib/k2hashfunc.cc:49-59); the
line also times the RCCL gather of every shard's hashes to rank 0 (shard.gather_hashes).
Every rank's shard is checked against the reference's digests
(tests/golden/digests.json, fixed32_1G chunks) outside the timed region.

At N = 1 the line also carries secondary results (configs 3, 4 and 5, config 2 with the fused
bucket index, RALLEDATA blobs, the k2himport TSV and mdbm scans + prehash of a file in HBM,
and the host-memory path) and a CPU baseline: the reference's own hash path (oracle/_ref),
timed on this host's cores.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config fixed32|csr|fixed4096|fixed32_1g|ralledata]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
# VALU issue roofline: every op of the FNV step (v_xor_b32_sdwa,
# v_mul_lo_u32, v_lshl_add_u32, v_mad_u64_u32, v_perm_b32) issues at ~4.19 cycles per wave64
# instruction per SIMD (profiles/r01_valu_rates.txt); 256 CUs x 4 SIMDs at the 2.4 GHz peak.
VALU_CYCLES_PER_INST = 4.19
VALU_SIMDS = 1024
VALU_PEAK_HZ = 2.4e9
FNV_OPS_PER_CHUNK = 86  # 16 bytes x 5 ops + 2 word pairs x 3 sign-smear ops (k2h_fnv_device.h)

KEYS_1G = 1 << 30
CONFIGS = {
    # name: (kind, keys per rank (None: 2^30 / world), key_len | (min,max), description)
    "fixed32": ("fixed", 1 << 24, 32, "16M x 32B fixed-length keys (BASELINE config 2)"),
    "csr": ("csr", 1 << 26, (8, 256), "64M mixed 8-256B keys, offsets+bytes CSR (BASELINE config 3)"),
    "fixed32_1g": ("fixed", None, 32, "2^30 x 32B keys sharded over the GPUs, RCCL gather of the hashes "
                                      "(BASELINE config 4)"),
    "fixed4096": ("fixed", 1 << 20, 4096, "1M x 4KiB keys (BASELINE config 5)"),
    # RALLEDATA blobs (hash + subhash + key + value) for a bulk direct set
    "ralledata": ("ralledata", 1 << 23, ((8, 64), (0, 256)),
                  "8M records (keys 8-64B, values 0-256B) -> RALLEDATA blobs with precomputed hashes"),
}
METRIC = "key hashes/sec + GiB/s (device-resident), batched 32B keys, 1 MI355X"


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--warm-ms", type=float, default=150.0,
                   help="keep warming up (untimed) until at least this much GPU time has passed: the "
                        "MI355X clock ramps over the first ~30 ms of back-to-back launches "
                        "(profiles/r01_clock_ramp.txt)")
    p.add_argument("--config", default=None, choices=sorted(CONFIGS),
                   help="default: fixed32 at N=1, fixed32_1g (config 4) at N>1")
    p.add_argument("--second", action="store_true", help="also emit the second hash (h2)")
    p.add_argument("--index", action="store_true",
                   help="fused bucket-index epilogue (kindex + ckindex outputs, SURVEY 8f rank 1) with a "
                        "2^28-slot table: cur_mask 0x0FFFFFFF, collision_mask 0xF")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-secondary", action="store_true", help="N=1: skip the secondary configs")
    p.add_argument("--no-verify", action="store_true", help="skip the digest checks")
    p.add_argument("--backend", default="nccl", help="torch.distributed backend for N>1 (nccl = RCCL)")
    p.add_argument("--dist", action="store_true",
                   help="initialise torch.distributed even at world size 1 (under torchrun): rehearses the "
                        "N>1 path -- RCCL init with device_id and timeout, barriers, the MAX all-reduce, "
                        "the gather -- on one GPU")
    p.add_argument("--rehearse-cpu", action="store_true",
                   help="no GPU: run the launcher / shard / gather path on CPU with the scalar plugin "
                        "(a rehearsal of the N>1 plumbing, not a measurement)")
    p.add_argument("--keys", type=int, default=0,
                   help="override the key count (tests / rehearsals): keys per rank for the weak configs, "
                        "the whole batch for the sharded ones (fixed32_1g; csr at N > 1 or with --dist)")
    p.add_argument("--child-timeout", type=float, default=540.0,
                   help="self-launcher: kill every rank after this long (below the driver's 600 s limit)")
    p.add_argument("--init-timeout", type=float, default=180.0,
                   help="torch.distributed init / collective timeout in seconds (N > 1)")
    p.add_argument("--inject-rank-failure", type=int, default=-1,
                   help="TEST ONLY: this rank exits with status 3 right after joining the process group "
                        "(exercises the launcher's fail-fast path)")
    return p.parse_args(argv)


# --------------------------------------------------------------------------------------
# Launcher: one fresh process per GPU (never an exec of this process)
# --------------------------------------------------------------------------------------
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(args) -> int:
    """Start args.gpus ranks of this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*),
    relay rank 0's stdout, return the worst exit code.  Runs before anything touches a
    GPU; the children are new processes (never an exec of this one).

    Fail-fast: every child is polled; the first rank that exits non-zero (or a run past
    --child-timeout) terminates the others, so a rank that dies in init or a collective
    ends the run with an error instead of leaving rank 0 blocked in RCCL until the
    driver's limit."""
    import tempfile

    port = _free_port()
    procs = []
    out0 = tempfile.TemporaryFile()  # rank 0's stdout (a file: no pipe to fill while we poll)
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:], env=env,
                                      stdout=out0 if r == 0 else subprocess.DEVNULL))
    print(f"launcher: rank pids {[p.pid for p in procs]}", file=sys.stderr, flush=True)
    deadline = time.monotonic() + args.child_timeout
    failed = None
    while True:
        rcs = [p.poll() for p in procs]
        bad = [(r, rc) for r, rc in enumerate(rcs) if rc not in (None, 0)]
        if bad:
            failed = f"rank {bad[0][0]} exited with {bad[0][1]}"
            break
        if all(rc == 0 for rc in rcs):
            break
        if time.monotonic() > deadline:
            failed = f"ranks still running after --child-timeout {args.child_timeout:.0f} s"
            break
        time.sleep(0.05)
    if failed:
        print(f"launcher: {failed}; terminating the other ranks", file=sys.stderr, flush=True)
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    out0.seek(0)
    sys.stdout.write(out0.read().decode(errors="replace"))
    sys.stdout.flush()
    if failed:
        return 1
    return max(abs(p.returncode) for p in procs)


# --------------------------------------------------------------------------------------
# Host description and the CPU baseline (rank 0, N = 1)
# --------------------------------------------------------------------------------------
def host_info() -> dict:
    info = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()
        info["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        info["cgroup_cpu_quota"] = None
    try:
        txt = Path("/proc/cpuinfo").read_text()
        names = [ln.split(":", 1)[1].strip() for ln in txt.splitlines() if ln.startswith("model name")]
        mhz = [float(ln.split(":", 1)[1]) for ln in txt.splitlines() if ln.startswith("cpu MHz")]
        info["model"] = names[0] if names else None
        info["mhz_now_avg"] = round(sum(mhz) / len(mhz), 1) if mhz else None
        mx = Path("/sys/devices/system/cpu/cpu0/cpufreq/cpuinfo_max_freq")
        info["mhz_max"] = int(mx.read_text()) / 1000 if mx.exists() else None
    except OSError:
        pass
    return info


def usable_cores(info: dict) -> int:
    n = info["affinity"]
    if info.get("cgroup_cpu_quota"):
        n = min(n, max(1, int(info["cgroup_cpu_quota"])))
    omp = os.environ.get("OMP_NUM_THREADS")  # the GPU box's per-GPU CPU share
    if omp and omp.isdigit():
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(keys_host, key_len: int, n: int) -> dict | None:
    """Reference hash path on the host cores (rank 0, N=1 only).  Bounded sample: the
    first n keys of the benchmark workload; best of 3 passes at 1 thread, at the usable
    cores and at every CPU the OS lists; worker threads are started and parked on a
    barrier before the clock starts (oracle/cpu_bench.c)."""
    import ctypes

    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle  # test/baseline infrastructure only

    lib = oracle.cpubench()
    so = str(oracle.REF_SO) if oracle.REF_SO.exists() else ""
    kind = "reference" if so else "port"
    info = host_info()
    cores = usable_cores(info)
    ptr = ctypes.c_void_p(keys_host.ctypes.data)
    dig = ctypes.c_uint64()

    def best(threads, m, inner=8, passes=3):  # seconds per pass over m keys, best of `passes`
        ts = [lib.cpu_bench_fixed(so.encode(), ptr, key_len, m, threads, inner, 0, ctypes.byref(dig))
              for _ in range(passes)]
        return min(ts) / inner if min(ts) > 0 else None

    m1 = min(n, 1 << 22)
    t1 = best(1, m1)
    tN = best(cores, n)
    tall = best(info["nproc"], n) if info["nproc"] and info["nproc"] != cores else tN
    # k2hbench `-type rw` hash path (BASELINE config 1): 100k loops x 10 scalar calls per
    # thread on 21-byte "KEY-%016X" keys; per-thread timing like tests/k2hbench.cc:937-976
    kb1 = min(lib.cpu_bench_k2hbench(so.encode(), 100000, 100000, 1, ctypes.byref(dig)) for _ in range(3))
    kbN = min(lib.cpu_bench_k2hbench(so.encode(), 100000, 100000, cores, ctypes.byref(dig)) for _ in range(3))
    nall = info["nproc"] or cores
    kbA = min(lib.cpu_bench_k2hbench(so.encode(), 100000, 100000, nall, ctypes.byref(dig)) for _ in range(3)) \
        if nall != cores else kbN
    if not (t1 and tN):
        return None
    # the reported value: the pass on the threads this process may use (the cgroup's CPU
    # share); the pass over every CPU the OS lists only time-shares that quota and is kept
    # as a sub-field
    threads, t = cores, tN
    kb = {"hash_calls_per_thread": 1000000,
          "threads_1": {"seconds": kb1, "calls_per_s": 1e6 / kb1 if kb1 > 0 else None},
          f"threads_{cores}": {"seconds": kbN, "calls_per_s": cores * 1e6 / kbN if kbN > 0 else None}}
    kb[f"threads_{nall}"] = {"seconds": kbA, "calls_per_s": nall * 1e6 / kbA if kbA > 0 else None}
    # the drop-in plugin (this repo's scalar k2h_hash / k2h_second_hash, libk2hfnv_plugin.so)
    # in the same harness, 1 thread: it must not be slower than the reference it replaces
    plugin = ROOT / "k2hash_amd" / "lib" / "libk2hfnv_plugin.so"
    drop_in = None
    if plugin.exists() and so:
        d_ref, d_plug = ctypes.c_uint64(), ctypes.c_uint64()
        tr = min(lib.cpu_bench_fixed(so.encode(), ptr, key_len, m1, 1, 8, 0, ctypes.byref(d_ref)) for _ in range(3)) / 8
        tp = min(lib.cpu_bench_fixed(str(plugin).encode(), ptr, key_len, m1, 1, 8, 0, ctypes.byref(d_plug))
                 for _ in range(3)) / 8
        kr = min(lib.cpu_bench_k2hbench(so.encode(), 100000, 100000, 1, ctypes.byref(d_ref)) for _ in range(3))
        kp = min(lib.cpu_bench_k2hbench(str(plugin).encode(), 100000, 100000, 1, ctypes.byref(d_plug))
                 for _ in range(3))
        drop_in = {"library": "k2hash_amd/lib/libk2hfnv_plugin.so", "threads": 1,
                   f"fixed{key_len}_keys_per_s": {"plugin": m1 / tp, "reference": m1 / tr},
                   "k2hbench_rw_calls_per_s": {"plugin": 1e6 / kp, "reference": 1e6 / kr},
                   "k2hbench_digest_equal": d_ref.value == d_plug.value}
    return {
        "value": n / t, "unit": "key hashes/s", "cores": threads, "kind": kind,
        "sample": f"first {n} keys of the same {key_len}B workload (first {m1} at 1 thread), h1 only, "
                  f"8 passes per run, best of 3 runs, on {threads} threads (the box's {cores}-CPU share; "
                  f"all {nall} listed CPUs in all_listed_cpus; reference lib/k2hashfunc.cc k2h_hash via dlsym)",
        "single_thread": m1 / t1,
        "cpu_share": {"threads": cores, "value": n / tN},
        "all_listed_cpus": {"threads": nall, "value": n / tall if tall else None},
        "host": info,
        "k2hbench_rw_100k": kb,
        "drop_in_plugin": drop_in,
    }


def cpu_baseline_workload(kind: str, host_bytes, host_off, key_len: int, n1: int, n: int, gpu_h1=None) -> dict:
    """The reference's k2h_hash (oracle/_ref via dlsym, else the C restatement) over a
    bounded prefix of a secondary config's exact input (SURVEY 8d CPU row ii):
    the first n1 keys on 1 thread and the first n keys on the usable cores (one shard of
    about equal bytes per parked worker thread), h1 only, best of 3 runs of `passes`
    passes.  key GB/s = key bytes hashed / s.  gpu_h1: the GPU's h1 of the same keys, checked
    against the CPU pass's xor-digest."""
    import ctypes

    import numpy as np

    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle  # test/baseline infrastructure only

    lib = oracle.cpubench()
    so = str(oracle.REF_SO) if oracle.REF_SO.exists() else ""
    info = host_info()
    cores = usable_cores(info)
    dig = ctypes.c_uint64()
    bptr = ctypes.c_void_p(host_bytes.ctypes.data)

    def run(m, threads, passes):
        if kind == "csr":
            optr = ctypes.c_void_p(host_off.ctypes.data)
            ts = [lib.cpu_bench_csr(so.encode(), bptr, optr, m, threads, passes, 0, ctypes.byref(dig)) for _ in range(3)]
            nbytes = int(host_off[m] - host_off[0])
        else:
            ts = [lib.cpu_bench_fixed(so.encode(), bptr, key_len, m, threads, passes, 0, ctypes.byref(dig))
                  for _ in range(3)]
            nbytes = m * key_len
        t = min(ts) / passes
        return {"threads": threads, "keys": m, "key_bytes": nbytes, "seconds_per_pass": t, "value": m / t,
                "key_gb_per_s": nbytes / t / 1e9}

    one = run(n1, 1, 2)
    many = run(n, cores, 2)
    res = {"kind": "reference" if so else "port", "unit": "key hashes/s", "single_thread": one, "cores": many,
           "value": many["value"], "cores_used": cores,
           "sample": f"first {n1} keys on 1 thread, first {n} keys on {cores} threads (the box's CPU share), "
                     "h1 only, 2 passes per run, best of 3 runs; reference lib/k2hashfunc.cc k2h_hash via dlsym"}
    if gpu_h1 is not None and kind == "csr":  # the CPU digest (one pass, n keys) against the GPU's hashes
        lib.cpu_bench_csr(so.encode(), bptr, ctypes.c_void_p(host_off.ctypes.data), n, 1, 1, 0, ctypes.byref(dig))
        res["digest_matches_gpu"] = int(np.bitwise_xor.reduce(gpu_h1.view(np.uint64))) == dig.value
    elif gpu_h1 is not None:
        lib.cpu_bench_fixed(so.encode(), bptr, key_len, n, 1, 1, 0, ctypes.byref(dig))
        res["digest_matches_gpu"] = int(np.bitwise_xor.reduce(gpu_h1.view(np.uint64))) == dig.value
    return res


# --------------------------------------------------------------------------------------
# Digests of the reference's outputs (tests/golden/digests.json): [xor, wrapping sum,
# wrapping sum of h*(2i+1)], i = global key index.  Computed on the device.
# --------------------------------------------------------------------------------------
def _golden():
    return json.loads((ROOT / "tests" / "golden" / "digests.json").read_text())["configs"]


def digest_dev(h, first: int) -> list[str]:
    return [f"{v:016x}" for v in digest_ints(h, first)]


def digest_ints(h, first: int) -> list[int]:
    """[xor, wrapping sum, wrapping sum of h * (2 i + 1)] of the hashes h of global keys
    first .. first + h.numel() - 1, as unsigned 64-bit ints.  Each term is a xor or a sum
    over keys, so the digest of a key range is the combination (xor, +, +) of the digests of
    any partition of it -- how sharded results are checked without gathering them."""
    import torch

    x = h
    while x.numel() > 1:
        half = x.numel() // 2
        y = x[:half] ^ x[half:2 * half]
        if x.numel() & 1:
            y[0] ^= x[-1]
        x = y
    xr = int(x[0].item()) if x.numel() else 0
    s = int(h.sum().item())
    w = 2 * (torch.arange(h.numel(), dtype=torch.int64, device=h.device) + first) + 1
    ws = int((h * w).sum().item())
    return [v & (2**64 - 1) for v in (xr, s, ws)]


def verify_sharded(h, first: int, chunks, dist=None, dev=None) -> dict:
    """Check reference chunks against hashes spread over the ranks: each rank digests the
    part of every chunk that lies in its key range [first, first + h.numel()) (zeros --
    the identity -- elsewhere), the parts are all-gathered and combined (xor, +, +) and
    every chunk wholly covered by the ranks is compared with the reference's digest.  Byte
    cuts (CSR) do not align with the reference's chunks, so no rank holds one whole."""
    import torch

    n = h.numel()
    parts = torch.zeros(len(chunks), 4, dtype=torch.int64)
    for j, c in enumerate(chunks):
        a, b = max(c["first"], first), min(c["first"] + c["count"], first + n)
        if a < b:
            d = digest_ints(h[a - first:b - first], a)
            parts[j, :3] = torch.tensor([v - (1 << 64) if v >= 1 << 63 else v for v in d], dtype=torch.int64)
            parts[j, 3] = b - a
    allp = [parts]
    if dist is not None and dist.is_initialized():
        gloo = dist.get_backend() == "gloo"
        mine = parts if gloo else parts.to(dev)
        allp = [torch.zeros_like(mine) for _ in range(dist.get_world_size())]
        dist.all_gather(allp, mine)
        allp = [t.cpu() for t in allp]
    ok, checked = True, 0
    for j, c in enumerate(chunks):
        xr = sm = ws = covered = 0
        for t in allp:
            v = [int(x) & (2**64 - 1) for x in t[j, :3].tolist()]
            xr ^= v[0]
            sm = (sm + v[1]) & (2**64 - 1)
            ws = (ws + v[2]) & (2**64 - 1)
            covered += int(t[j, 3])
        if covered == c["count"]:
            ok &= [f"{v:016x}" for v in (xr, sm, ws)] == c["h1"]
            checked += 1
    return {"chunks_checked": checked, "ok": bool(ok) and checked > 0, "ranks": len(allp),
            "how": "per-rank partial digests of every reference chunk, all-gathered and combined"}


def verify_chunks(h, first: int, chunks) -> dict:
    """Check every reference chunk that lies wholly inside [first, first + h.numel())."""
    ok, checked = True, 0
    for c in chunks:
        a, b = c["first"], c["first"] + c["count"]
        if a >= first and b <= first + h.numel():
            ok &= digest_dev(h[a - first:b - first], a) == c["h1"]
            checked += 1
    return {"chunks_checked": checked, "ok": bool(ok)}


def golden_chunks(kind: str, shape, total: int):
    """The reference digests' chunks for a whole workload of `total` keys of this kind
    (tests/golden/digests.json), or None when the reference has none at that size."""
    for g in _golden().values():
        if g["n"] != total or g["kind"] != kind:
            continue
        if (kind == "fixed" and g["key_len"] == shape) or (kind == "csr" and (g["min_len"], g["max_len"]) == tuple(shape)):
            return g.get("chunks") or [dict(first=0, count=g["n"], h1=g["h1"])]
    return None


def measure_gather(h, counts, step, gsteps: int, dist, dev, sync=lambda: None) -> tuple[dict, object]:
    """The path's one exchange: every rank's hashes to rank 0 (shard.gather_hashes,
    RCCL point-to-point over xGMI, or gloo), timed alone and back to back with the hash step.
    Max over ranks.  Returns (the line's `gather` object without verify_root, rank 0's result)."""
    import torch

    from k2hash_amd import shard

    res = None
    for _ in range(2):
        res = shard.gather_hashes(h, counts=counts)
    sync()
    dist.barrier()
    g0 = time.perf_counter()
    for _ in range(gsteps):
        res = shard.gather_hashes(h, counts=counts)
    sync()
    dist.barrier()
    gs = torch.tensor([(time.perf_counter() - g0) / gsteps], dtype=torch.float64, device=dev)
    dist.all_reduce(gs, op=dist.ReduceOp.MAX)
    gather_s = float(gs.item())
    dist.barrier()  # hash + gather back to back (the end-to-end step of a bulk loader)
    sync()
    c0 = time.perf_counter()
    for _ in range(gsteps):
        step(0)
        res = shard.gather_hashes(h, counts=counts)
    sync()
    dist.barrier()
    cs = torch.tensor([(time.perf_counter() - c0) / gsteps], dtype=torch.float64, device=dev)
    dist.all_reduce(cs, op=dist.ReduceOp.MAX)
    combo_s = float(cs.item())
    to_root = 8 * (sum(counts) - counts[0])
    return {"backend": dist.get_backend(), "counts": list(counts), "ms_per_gather": gather_s * 1e3,
            "bytes_to_root": to_root, "root_recv_gb_per_s": to_root / gather_s / 1e9,
            "p2p_peers_at_root": sum(1 for c in counts[1:] if c),
            "with_gather": {"ms_per_step": combo_s * 1e3, "value": sum(counts) / combo_s,
                            "unit": "key hashes/s (hashed and gathered at rank 0)"}}, res


# --------------------------------------------------------------------------------------
# Timing
# --------------------------------------------------------------------------------------
_ROCTX = []


def _roctx():
    """rocprofiler-sdk's roctx, loaded only when K2H_BENCH_MARKERS=1 (tools/profile_line.sh
    runs the driver's own command under rocprofv3 --kernel-trace --marker-trace with it): the
    timed region of every line entry becomes a named range, so each figure in the line is
    recomputed from the kernels inside its range (tools/summarize_line_profile.py)."""
    if not _ROCTX:
        lib = None
        if os.environ.get("K2H_BENCH_MARKERS") == "1":
            import ctypes

            lib = ctypes.CDLL("librocprofiler-sdk-roctx.so.1")
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
        _ROCTX.append(lib)
    return _ROCTX[0]


def timed(step, steps: int, warmup: int, warm_ms: float, world: int = 1, dist=None, dev=None,
          label: str = "headline"):
    """W untimed launches, then warm up for >= warm_ms, then EXACTLY `steps` launches bracketed
    by barrier + synchronize.  Returns (wall seconds (max over ranks), average launch time from
    one event pair on the launch stream, extra warm-up launches).  With K2H_BENCH_MARKERS=1 the
    synchronised timed region is the roctx range "timed:<label>"."""
    import torch

    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    w0, extra = time.perf_counter(), 0
    while (time.perf_counter() - w0) * 1e3 < warm_ms:
        for i in range(10):
            step(i)
        extra += 10
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    distributed = dist is not None and dist.is_initialized()  # (N > 1, or --dist at N = 1)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    mk = _roctx()
    if mk:
        mk.roctxRangePushA(f"timed:{label}".encode())
    t0 = time.perf_counter()
    e0.record()
    for i in range(steps):
        step(i)
    e1.record()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if mk:
        mk.roctxRangePop()
    if distributed:
        dist.barrier()
    elapsed = t1 - t0
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, e0.elapsed_time(e1) / steps / 1e3, extra


def _profile(kind: str, name: str, keys: int | None):
    """profiles/<kind>_<name>.json scaled to a launch of `keys` keys: the counts are per
    launch of the kernel over `keys_per_launch` keys, and every per-key quantity of these
    kernels (instructions, bytes) is linear in the key count.  None when the profile is
    missing or was not taken per key."""
    prof = ROOT / "profiles" / f"{kind}_{name}.json"
    if not prof.exists():
        return None, None
    d = json.loads(prof.read_text())
    per = d.get("keys_per_launch")
    if not per or not keys:
        return None, None
    return d, keys / per


def valu_fields(name: str, kern_s: float, model_insts: float, keys: int | None = None) -> dict:
    """VALU-issue roofline: wave64 VALU instructions per launch (rocprofv3 SQ_INSTS_VALU pass,
    profiles/valu_<name>.json scaled to this launch's key count, else the FNV-step model) at
    the peak issue rate, over the measured launch time."""
    insts, src = model_insts, "model: 86 slow-issue VALU ops per 16-byte chunk per 64 keys"
    d, scale = _profile("valu", name, keys)
    if d is not None:
        insts = float(d["valu_insts_per_launch"]) * scale
        src = (f"profiles/valu_{name}.json ({d.get('round', '')}; {d['keys_per_launch']} keys per profiled launch, "
               f"scaled x{scale:.4g} to this launch)")
    floor_s = insts * VALU_CYCLES_PER_INST / (VALU_SIMDS * VALU_PEAK_HZ)
    r = {"valu_frac": floor_s / kern_s, "valu_insts_per_launch": insts, "valu_floor_us": floor_s * 1e6,
         "valu_source": src}
    return r


def traffic_of(name: str, keys: int | None = None):
    """HBM bytes per launch from the PMC pass (profiles/traffic_<name>.json), scaled to this
    launch's key count; None without a per-key profile."""
    d, scale = _profile("traffic", name, keys)
    return None if d is None else d["hbm_bytes_per_launch"] * scale


def roofline(name: str, algo_bytes: int, kern_s: float, model_insts: float, keys: int | None = None) -> dict:
    achieved = algo_bytes / kern_s / 1e9
    r = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
         "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic_of(name, keys), "algorithmic_bytes_per_launch": algo_bytes,
         "keys_per_launch": keys}
    r.update(valu_fields(name, kern_s, model_insts, keys))
    return r


def chunks_of(length: int) -> int:
    return (length + 15) // 16


# --------------------------------------------------------------------------------------
# Secondary results at N = 1 (configs 3, 4, 5, SURVEY 8f rows 1-3 and the host-memory path)
# --------------------------------------------------------------------------------------
def secondary_csr(dev, steps, warm_ms, verify, cpu=False):
    import numpy as np
    import torch

    import k2hash_amd
    from k2hash_amd import batch

    n, (lo, hi) = CONFIGS["csr"][1], CONFIGS["csr"][2]
    off = batch.synth_offsets(n, dev, lo, hi)
    nbytes = int(off[-1].item())
    data = batch.synth_bytes(nbytes, dev)
    h1 = torch.empty(n, dtype=torch.int64, device=dev)
    wall, kern, _ = timed(lambda i: k2hash_amd.hash_csr(data, off, out=(h1, None)), steps, 3, warm_ms,
                          label="csr")
    algo = nbytes + 8 * n + 8 * (n + 1)
    model = sum(chunks_of(L) for L in range(lo, hi + 1)) / (hi - lo + 1) * FNV_OPS_PER_CHUNK * n / 64
    res = {"workload": CONFIGS["csr"][3], "keys": n, "steps": steps, "ms_per_step": wall / steps * 1e3, "kernel_ms": kern * 1e3,
           "value": n * steps / wall, "unit": "key hashes/s", "roofline": roofline("csr", algo, kern, model, n)}
    if verify:
        res["verify"] = verify_chunks(h1, 0, _golden()["csr_8_256_64M"]["chunks"])
    if cpu:  # the reference on the host cores over the first 16M keys of the same input
        m = 1 << 24
        host_off = off[:m + 1].cpu().numpy().view(np.uint64)
        host_bytes = data[:int(host_off[-1])].cpu().numpy()
        res["cpu_baseline"] = cpu_baseline_workload("csr", host_bytes, host_off, 0, 1 << 21, m,
                                                    h1[:m].cpu().numpy())
        res["gpu_over_cpu_cores"] = res["value"] / res["cpu_baseline"]["value"]
        del host_off, host_bytes
    del off, data, h1
    torch.cuda.empty_cache()
    return res


def secondary_fixed(name, dev, steps, warm_ms, verify, golden_name, cpu=False):
    import numpy as np
    import torch

    import k2hash_amd
    from k2hash_amd import batch

    _, n, L, desc = CONFIGS[name]
    n = n or KEYS_1G
    keys = batch.synth_bytes(n * L, dev)
    h1 = torch.empty(n, dtype=torch.int64, device=dev)
    wall, kern, _ = timed(lambda i: k2hash_amd.hash_fixed(keys, L, out=(h1, None)), steps, 3, warm_ms,
                          label=name)
    algo = n * L + 8 * n
    model = n / 64 * chunks_of(L) * FNV_OPS_PER_CHUNK
    res = {"workload": desc + (" -- all 2^30 keys on one GPU" if name == "fixed32_1g" else ""), "keys": n,
           "steps": steps, "ms_per_step": wall / steps * 1e3, "kernel_ms": kern * 1e3, "value": n * steps / wall,
           "unit": "key hashes/s", "key_gib_per_s": n * L * steps / wall / 2**30,
           "roofline": roofline(name, algo, kern, model, n)}
    if verify:
        g = _golden()[golden_name]
        res["verify"] = verify_chunks(h1, 0, g.get("chunks") or [dict(first=0, count=g["n"], h1=g["h1"])])
    if cpu:  # the reference on the host cores over a prefix of the same keys (1 GiB)
        m = min(n, (1 << 30) // L)
        host = keys[:m * L].cpu().numpy()
        res["cpu_baseline"] = cpu_baseline_workload("fixed", host, None, L, max(1, m // 8), m,
                                                    h1[:m].cpu().numpy())
        res["gpu_over_cpu_cores"] = res["value"] / res["cpu_baseline"]["value"]
        del host
    del keys, h1
    torch.cuda.empty_cache()
    return res


def secondary_index(dev, steps, warm_ms, verify):
    """config 2 with the bucket-index epilogue fused into the hash kernel
    (kindex / ckindex per key, lib/k2hshm.cc:810-833, 1093); checked against
    tests/golden/index_digest.json (oracle hash + oracle bucket index)."""
    import torch

    from k2hash_amd import batch

    _, n, L, desc = CONFIGS["fixed32"]
    g = json.loads((ROOT / "tests" / "golden" / "index_digest.json").read_text())
    sets = [batch.synth_bytes(n * L, dev, byte_off=s * n * L) for s in range(2)]  # set 0 = the digest's keys
    out = [torch.empty(n, dtype=torch.int64, device=dev) for _ in range(3)]
    wall, kern, _ = timed(lambda i: batch.hash_fixed_index(sets[i % 2], L, g["cur_mask"], g["collision_mask"],
                                                           out=(out[0], None, out[1], out[2])), steps, 3, warm_ms,
                          label="fixed32_index")
    algo = n * L + 8 * n + 16 * n
    model = n / 64 * chunks_of(L) * FNV_OPS_PER_CHUNK
    res = {"workload": desc + " + fused bucket index (cur_mask 2^28-1, collision_mask 0xF)", "keys": n,
           "steps": steps, "ms_per_step": wall / steps * 1e3, "kernel_ms": kern * 1e3, "value": n * steps / wall,
           "unit": "key hashes + bucket positions/s", "roofline": roofline("fixed32_index", algo, kern, model, n)}
    if verify:
        batch.hash_fixed_index(sets[0], L, g["cur_mask"], g["collision_mask"], out=(out[0], None, out[1], out[2]))
        ok = digest_dev(out[0], 0) == g["h1"] and digest_dev(out[1], 0) == g["kindex"] and \
            digest_dev(out[2], 0) == g["ckindex"]
        res["verify"] = {"ok": ok, "against": "tests/golden/index_digest.json"}
    del sets, out
    torch.cuda.empty_cache()
    return res


def ralledata_set(dev, n: int, s: int, first: int = 0, world: int = 1, rank: int = 0):
    """Input set s of bench's RALLEDATA workload for this rank: 8M records (keys 8-64 B,
    values 0-256 B), key and value lengths from the records' global indices, bytes from
    disjoint splitmix64 streams.  Set 0 of rank 0 is tests/golden/ralledata_digest.json's
    workload.  Returns ((keys, key_off, vals, val_off), (blob, blob_off), total blob bytes);
    the blob is zero-padded to whole 8-byte words (the digest is taken over u64 words)."""
    import torch

    from k2hash_amd import batch

    (klo, khi), (vlo, vhi) = CONFIGS["ralledata"][2]
    base = first + s * world * n
    ko = batch.synth_offsets(n, dev, klo, khi, first_key=base)
    vo = batch.synth_offsets(n, dev, vlo, vhi, seed=batch.SEED_LENS + 7, first_key=base)
    kb, vb = int(ko[-1].item()), int(vo[-1].item())
    kd = batch.synth_bytes(kb, dev, byte_off=s * (1 << 36) + rank * (1 << 34))
    vd = batch.synth_bytes(vb, dev, byte_off=s * (1 << 36) + rank * (1 << 34) + (1 << 33))
    total = 80 * n + kb + vb
    blob = torch.zeros((total + 7) // 8 * 8, dtype=torch.uint8, device=dev)
    boff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    return (kd, ko, vd, vo), (blob, boff), total


def ralledata_algo_bytes(io) -> int:
    """Minimal traffic of one build: key + value bytes and their offsets in, the blobs and
    blob offsets out."""
    (kd, ko, vd, vo) = io
    n = ko.numel() - 1
    kb, vb = kd.numel(), vd.numel()
    return (kb + vb + 16 * (n + 1)) + (80 * n + kb + vb + 8 * (n + 1))


def secondary_ralledata(dev, steps, warm_ms, verify):
    """RALLEDATA blobs (hash + subhash + lengths + key + value) for bench's
    ralledata workload, one kernel per call, two input sets rotated exactly as the standalone
    `--config ralledata` run (the line's figure and the profile's are the same
    code path); checked against tests/golden/ralledata_digest.json (the oracle's layout
    restatement over the reference-pinned hash)."""
    import torch

    from k2hash_amd import ralledata

    _, n, ((klo, khi), _v), desc = CONFIGS["ralledata"]
    sets = [ralledata_set(dev, n, s) for s in range(2)]

    def step(i):
        (kd, ko, vd, vo), (blob, boff), total = sets[i % 2]
        ralledata.build_ralledata(kd, ko, vd, vo, out=blob, blob_off=boff, total=total)

    wall, kern, _ = timed(step, steps, 3, warm_ms, label="ralledata")
    algo = max(ralledata_algo_bytes(io) for io, _o, _t in sets)
    total = sets[0][2]
    model = sum(chunks_of(L) for L in range(klo, khi + 1)) / (khi - klo + 1) * FNV_OPS_PER_CHUNK * n / 64
    res = {"workload": desc, "records": n, "steps": steps, "ms_per_step": wall / steps * 1e3, "kernel_ms": kern * 1e3,
           "value": n * steps / wall, "unit": "records/s", "blob_gb_per_s": total * steps / wall / 1e9,
           "input_sets": 2, "roofline": roofline("ralledata", algo, kern, model, n)}
    if verify:
        (_io, (blob, boff), total) = sets[0]  # written by step 18, untouched since
        g = json.loads((ROOT / "tests" / "golden" / "ralledata_digest.json").read_text())
        ok = g["n"] == n and g["bytes"] == total and digest_dev(blob.view(torch.int64), 0) == g["blob"] and \
            digest_dev(boff, 0) == g["blob_off"]
        res["verify"] = {"ok": ok, "against": "tests/golden/ralledata_digest.json"}
    del sets
    torch.cuda.empty_cache()
    return res


IMPORT_N, IMPORT_KEY_LENS, IMPORT_VAL_LENS, IMPORT_BYTE_OFF = 1 << 23, (8, 64), (0, 200), 1 << 34


def import_workload(dev):
    """bench's k2himport TSV workload, built on the device: 2^23 records "key TAB value
    NEWLINE" (key lengths 8-64, value lengths 0-200, printable bytes) -- the file
    tests/golden/make_import_digest.py builds on the host from the same generators."""
    import torch

    from k2hash_amd import batch

    n = IMPORT_N
    kl = batch.synth_offsets(n, dev, *IMPORT_KEY_LENS, seed=batch.SEED_LENS + 11).diff()
    vl = batch.synth_offsets(n, dev, *IMPORT_VAL_LENS, seed=batch.SEED_LENS + 13).diff()
    off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(kl + vl + 2, dim=0, out=off[1:])
    data = batch.synth_bytes(int(off[-1].item()), dev, byte_off=IMPORT_BYTE_OFF)
    data.remainder_(95).add_(32)
    data[off[:-1] + kl] = 9
    data[off[1:] - 1] = 10
    return data


def secondary_import(dev, steps, warm_ms, verify):
    """k2himport's TSV loop (tests/k2himport.cc:81-86) over a file resident
    in HBM -- records (key / value offsets and C-string lengths) and every key's h1 / h2 as
    K2HShm::Set(const char*) hashes it, from one call (k2h_amd_import_scan_prehash_device,
    which synchronises its stream: the step time is the call's wall time).  Checked against
    tests/golden/import_digest.json (the tool's own getline loop + the reference hash)."""
    import torch

    from k2hash_amd import archive

    data = import_workload(dev)
    n, size = IMPORT_N, data.numel()
    out = {}

    def step(i):
        out["r"] = archive.import_scan_prehash_device(data)

    wall, kern, _ = timed(step, steps, 2, warm_ms, label="import")
    algo = size + 32 * n + 16 * n  # the file once, the records, the two hashes
    model = sum(chunks_of(L) for L in range(IMPORT_KEY_LENS[0], IMPORT_KEY_LENS[1] + 1)) / \
        (IMPORT_KEY_LENS[1] - IMPORT_KEY_LENS[0] + 1) * FNV_OPS_PER_CHUNK * n / 64
    res = {"workload": f"{n} TSV records (keys 8-64 B, values 0-200 B, {size} B file in HBM) -> records + h1/h2",
           "records": n, "file_bytes": size, "steps": steps, "ms_per_step": wall / steps * 1e3, "kernel_ms": kern * 1e3,
           "value": n * steps / wall, "unit": "records/s", "file_gb_per_s": size * steps / wall / 1e9,
           "roofline": roofline("import", algo, wall / steps, model, n)}
    if verify:
        res["verify"] = _import_verify(out["r"], "import_digest.json")
    del data, out
    torch.cuda.empty_cache()
    return res


MDBM_HDR = b"format=print\ntype=btree\nmdbm_pagesize=4096\nmdbm_pagecount=1\nHEADER=END\n"


def import_mdbm_workload(dev):
    """The import workload's 2^23 records in mdbm's print format (tests/k2himport.cc:95-117):
    the five header lines, then a key line and a value line per record, built on the device
    -- the file tests/golden/make_import_digest.py --mdbm builds on the host.  Returns the
    file and each record's (key_off, key_len, val_off, val_len) by construction."""
    import torch

    from k2hash_amd import batch

    n = IMPORT_N
    kl = batch.synth_offsets(n, dev, *IMPORT_KEY_LENS, seed=batch.SEED_LENS + 11).diff()
    vl = batch.synth_offsets(n, dev, *IMPORT_VAL_LENS, seed=batch.SEED_LENS + 13).diff()
    h = len(MDBM_HDR)
    off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(kl + vl + 2, dim=0, out=off[1:])
    off += h
    data = batch.synth_bytes(int(off[-1].item()), dev, byte_off=IMPORT_BYTE_OFF)
    data.remainder_(95).add_(32)
    data[:h] = torch.frombuffer(bytearray(MDBM_HDR), dtype=torch.uint8).to(dev)
    data[off[:-1] + kl] = 10
    data[off[1:] - 1] = 10
    exp = torch.stack([off[:-1], kl, off[:-1] + kl + 1, vl], dim=1)
    return data, exp


def _import_verify(out, golden: str) -> dict:
    import torch  # noqa: F401

    recs, h1, h2 = out
    g = json.loads((ROOT / "tests" / "golden" / golden).read_text())
    cols = {"key_off": recs[:, 0], "key_len": recs[:, 1], "val_off": recs[:, 2], "val_len": recs[:, 3],
            "h1": h1, "h2": h2}
    ok = g["records"] == recs.shape[0] == IMPORT_N and all(digest_dev(v.contiguous(), 0) == g[k]
                                                           for k, v in cols.items())
    return {"ok": bool(ok), "against": f"tests/golden/{golden}"}


def secondary_import_mdbm(dev, steps, warm_ms, verify):
    """SURVEY 8f row 3, mdbm form: k2himport's mdbm loop (tests/k2himport.cc:95-117: the
    HEADER=END check, then key line / value line) over the import workload's records in
    mdbm's print format, resident in HBM -> records + every key's h1 / h2, one call
    (k2h_amd_import_scan_prehash_device, format mdbm).  Checked against
    tests/golden/import_mdbm_digest.json (the tool's getline loop + the reference hash)."""
    import torch

    from k2hash_amd import archive

    data, _exp = import_mdbm_workload(dev)
    del _exp
    n, size = IMPORT_N, data.numel()
    out = {}

    def step(i):
        out["r"] = archive.import_scan_prehash_device(data, "mdbm")

    wall, kern, _ = timed(step, steps, 2, warm_ms, label="import_mdbm")
    algo = size + 32 * n + 16 * n
    model = sum(chunks_of(L) for L in range(IMPORT_KEY_LENS[0], IMPORT_KEY_LENS[1] + 1)) / \
        (IMPORT_KEY_LENS[1] - IMPORT_KEY_LENS[0] + 1) * FNV_OPS_PER_CHUNK * n / 64
    res = {"workload": f"{n} mdbm records (key line 8-64 B, value line 0-200 B, {size} B file in HBM) -> "
                       "records + h1/h2",
           "records": n, "file_bytes": size, "steps": steps, "ms_per_step": wall / steps * 1e3, "kernel_ms": kern * 1e3,
           "value": n * steps / wall, "unit": "records/s", "file_gb_per_s": size * steps / wall / 1e9,
           "roofline": roofline("import_mdbm", algo, wall / steps, model, n)}
    if verify:
        res["verify"] = _import_verify(out["r"], "import_mdbm_digest.json")
    del data, out
    torch.cuda.empty_cache()
    return res


def secondary_host(dev, reps=5):
    """Host-memory path (PCIe-inclusive; never `value`): keys in pageable host memory ->
    k2h_amd_hash_*_host -> hashes in host memory.  16M x 32 B fixed keys, and 8M CSR keys
    of config 3's length mix (1/8 of it).  Best / median over `reps` calls on one buffer,
    and one call on a freshly written buffer the HIP runtime has never seen."""
    import numpy as np
    import torch

    import k2hash_amd
    from k2hash_amd import batch

    def run(fn, fresh_fn, moved, n, golden, first_key=0):
        """fn(inp, out): out=None allocates the hash arrays (first-touch page faults of fresh
        memory inside the call); timed best of `reps` with a reused output array."""
        h1 = np.empty(n, np.uint64)
        ts, tn = [], []
        for r in range(reps + 1):
            t0 = time.perf_counter()
            fn(None, h1)
            if r:
                ts.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            fn(None, None)
            tn.append(time.perf_counter() - t0)
        fresh = fresh_fn()
        t0 = time.perf_counter()
        fn(fresh, None)
        t_fresh = time.perf_counter() - t0
        t = min(ts)
        ok = verify_chunks(torch.from_numpy(h1.view(np.int64)), first_key, golden)["ok"]
        return {"keys": n, "ms_per_call_best": t * 1e3, "ms_per_call_median": sorted(ts)[len(ts) // 2] * 1e3,
                "ms_new_output_array": min(tn) * 1e3, "ms_fresh_input_and_output": t_fresh * 1e3,
                "value": n / t, "unit": "key hashes/s", "moved_gb_per_s": moved / t / 1e9, "verify_ok": ok}

    n, L = CONFIGS["fixed32"][1], 32
    keys = batch.synth_bytes(n * L, dev).cpu().numpy()
    g = _golden()["fixed32_16M"]
    fixed = run(lambda k, o: k2hash_amd.hash_fixed_host(keys if k is None else k, L,
                                                        out=None if o is None else (o, None)),
                lambda: keys.copy(), n * L + 8 * n, n, [dict(first=0, count=n, h1=g["h1"])])
    fixed["workload"] = "16M x 32B keys, pageable host memory in and out (k2h_amd_hash_fixed_host)"
    m = 1 << 23
    off_d = batch.synth_offsets(m, dev, 8, 256)
    data = batch.synth_bytes(int(off_d[-1].item()), dev).cpu().numpy()
    off = off_d.cpu().numpy().astype(np.uint64)
    del off_d
    gc = _golden()["csr_8_256_64M"]["chunks"]
    csr = run(lambda d, o: k2hash_amd.hash_csr_host(data if d is None else d, off,
                                                    out=None if o is None else (o, None)),
              lambda: data.copy(), data.size + 8 * (m + 1) + 8 * m, m, gc)
    csr["workload"] = "8M CSR keys of 8-256B (the first 8M of config 3), pageable host memory (k2h_amd_hash_csr_host)"
    torch.cuda.empty_cache()
    return {"fixed32": fixed, "csr_8M": csr}


# --------------------------------------------------------------------------------------
# Rehearsal of the N > 1 plumbing without a GPU (scalar plugin hashes, gloo gather)
# --------------------------------------------------------------------------------------
def rehearse_cpu(args, world, rank):
    """The N > 1 path without a GPU: the same sharding (equal key counts for fixed keys,
    byte cuts of one CSR batch for --config csr), the same barrier-bracketed timing and MAX
    all-reduce, the same gather measurement (measure_gather: counts, bytes_to_root, one
    point-to-point receive per peer at the root) and the same sharded digest check
    (verify_sharded), over gloo, with the scalar plugin hashing each rank's keys."""
    import numpy as np
    import torch
    import torch.distributed as dist

    import k2hash_amd
    from k2hash_amd import shard

    import datetime

    dist.init_process_group(args.backend if args.backend != "nccl" else "gloo",
                            timeout=datetime.timedelta(seconds=args.init_timeout))
    if rank == args.inject_rank_failure:
        os._exit(3)  # TEST ONLY (--inject-rank-failure): die before the first collective
    csr = args.config == "csr"
    total = args.keys or 4096
    rng = np.random.default_rng(1234)
    if csr:  # one batch of 8-256 B keys (plus some empty ones), cut by bytes
        lens = rng.integers(8, 257, size=total)
        lens[::61] = 0
        offs = np.zeros(total + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        cuts = shard.csr_cuts(offs, world)
        raw = rng.integers(0, 256, size=int(offs[-1]), dtype=np.uint8)
        keys = [raw[offs[i]:offs[i + 1]].tobytes() for i in range(total)]
    else:
        cuts = [shard.shard_range(total, r, world) for r in range(world)]
        raw = rng.integers(0, 256, size=total * 32, dtype=np.uint8)
        keys = [raw[i * 32:(i + 1) * 32].tobytes() for i in range(total)]
    first, last = cuts[rank]
    mine = keys[first:last]
    h = None

    def step(_):
        nonlocal h
        h = torch.tensor([k2hash_amd.k2h_hash(k) for k in mine], dtype=torch.uint64).view(torch.int64)

    for i in range(args.warmup):
        step(i)
    step(0)
    dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    # the reference chunks here: the oracle-free product scalar hash over 4 equal key ranges
    ref = [k2hash_amd.k2h_hash(k) for k in keys]
    ref_t = torch.tensor(ref, dtype=torch.uint64).view(torch.int64)
    q = max(1, total // 4)
    chunks = [dict(first=a, count=min(q, total - a), h1=digest_dev(ref_t[a:a + q], a)) for a in range(0, total, q)]
    verify = verify_sharded(h, first, chunks, dist)
    counts = [b - a for a, b in cuts]
    gather, res = measure_gather(h, counts, step, 2, dist, None)
    if rank == 0:
        ok = res.view(torch.uint64).tolist() == ref
        gather["ok"] = ok
        gather["verify_root"] = verify_chunks(res, 0, chunks)
        if csr:
            gather["shard_key_bytes"] = [int(offs[b] - offs[a]) for a, b in cuts]
        print(json.dumps({"metric": METRIC, "value": total * args.steps / float(el.item()), "unit": "key hashes/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": float(el.item()) / args.steps * 1e3, "higher_is_better": True,
                          "scaling": "strong", "vs_baseline": None, "dtype": "u64 (u8 key bytes in)",
                          "data": "synthetic", "device": "cpu rehearsal (scalar plugin; NOT a measurement)",
                          "config": {"workload": (f"one batch of {total} CSR keys cut by bytes over {world} ranks"
                                                  if csr else f"{total} x 32B keys sharded over {world} ranks"),
                                     "keys_total": total, "parallelism": f"shard{world}"},
                          "verify": verify, "gather": gather}), flush=True)
    dist.destroy_process_group()


# --------------------------------------------------------------------------------------
def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args))  # before anything touches a GPU
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.rehearse_cpu:
        return rehearse_cpu(args, world, rank)

    import torch
    import torch.distributed as dist

    import k2hash_amd
    from k2hash_amd import batch, shard

    name = args.config or ("fixed32" if world == 1 else "fixed32_1g")
    kind, n, shape, desc = CONFIGS[name]
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(ndev, 1))  # one process per GPU; wraps only in rehearsals
    torch.cuda.set_device(dev)
    use_dist = world > 1 or args.dist
    if use_dist:
        import datetime

        tmo = datetime.timedelta(seconds=args.init_timeout)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=tmo)
        else:
            dist.init_process_group(args.backend, timeout=tmo)
        if rank == args.inject_rank_failure:
            os._exit(3)  # TEST ONLY (--inject-rank-failure): die before the first collective

    # --- synthetic input: this rank's global key range -----------------------------------
    # Sharded configs (strong scaling, one batch over the ranks): config 4 (fixed32_1g, 2^30
    # keys, equal key counts) and, at N > 1 or with --dist, config 3 (csr: ONE batch of 2^26
    # keys cut by BYTES, SURVEY 8e -- shard.csr_cuts over the batch's offsets, each rank's
    # offsets rebased to its own bytes).  Weak configs: every rank its own batch of n keys.
    strong = n is None or (kind == "csr" and use_dist)
    cuts = None
    total = None
    if strong:
        total = args.keys or (KEYS_1G if n is None else n)
        if kind == "csr":
            # The byte cuts once, on rank 0 (the whole batch's offsets: 2^26 + 1 int64), then
            # broadcast as the world + 1 key cuts and their byte offsets; every rank then
            # synthesises only its own keys' offsets (a key's length is a function of its
            # index), rebased to its first byte (each rank built the whole array).
            plan = torch.zeros(2 * (world + 1), dtype=torch.int64,
                               device=dev if args.backend == "nccl" else "cpu")
            if rank == 0:
                off_g = batch.synth_offsets(total, dev, shape[0], shape[1])
                ks = [a for a, _ in shard.csr_cuts(off_g, world)] + [total]
                plan.copy_(torch.tensor(ks + [int(off_g[k].item()) for k in ks], dtype=torch.int64))
                del off_g
            if world > 1:
                dist.broadcast(plan, 0)
            ks, bs = plan[:world + 1].tolist(), plan[world + 1:].tolist()
            cuts = [(ks[r], ks[r + 1]) for r in range(world)]
            cut_bytes = [bs[r + 1] - bs[r] for r in range(world)]
            first, last = cuts[rank]
        else:
            first, last = shard.shard_range(total, rank, world)
        n = last - first
    else:
        first = rank * n
        if args.keys:
            n = args.keys
    nsets = 1 if strong else 2  # sharded batches (config 4: >= 4 GiB per rank) dwarf the 256 MiB Infinity Cache
    sets, algo_bytes, key_bytes = [], 0, 0
    for s in range(nsets):
        base = first + s * world * n  # set 0 is the rank's shard of the reference workload
        if kind == "fixed":
            sets.append((batch.synth_bytes(n * shape, dev, byte_off=base * shape), None))
            algo_bytes, key_bytes = n * shape + 8 * n, n * shape
        elif kind == "ralledata":  # the same sets as secondary_ralledata (ralledata_set)
            io, outb, tot = ralledata_set(dev, n, s, first, world, rank)
            sets.append((io, outb + (tot,)))
            algo_bytes = max(algo_bytes, ralledata_algo_bytes(io))
            key_bytes = max(key_bytes, io[0].numel())
        elif strong:  # this rank's byte range of the one reference batch (byte stream offset = its first byte)
            off = batch.synth_offsets(last - first, dev, shape[0], shape[1], first_key=first)
            b0 = bs[rank]
            nb = int(off[-1].item())
            data = batch.synth_bytes(nb, dev, byte_off=b0)
            sets.append((data, off))
            algo_bytes, key_bytes = nb + 8 * n + 8 * (n + 1), nb
        else:
            off = batch.synth_offsets(n, dev, shape[0], shape[1], first_key=base)
            nb = int(off[-1].item())
            data = batch.synth_bytes(nb, dev, byte_off=s * (1 << 36) + rank * (1 << 34))
            sets.append((data, off))
            algo_bytes, key_bytes = max(algo_bytes, nb + 8 * n + 8 * (n + 1)), max(key_bytes, nb)
    if args.second:
        algo_bytes += 8 * n
    if args.index:
        algo_bytes += 16 * n  # kindex + ckindex writes
    outs = [(torch.empty(n, dtype=torch.int64, device=dev),
             torch.empty(n, dtype=torch.int64, device=dev) if args.second else None) for _ in range(nsets)]
    idx = [(torch.empty(n, dtype=torch.int64, device=dev), torch.empty(n, dtype=torch.int64, device=dev))
           for _ in range(nsets)] if args.index else None
    torch.cuda.synchronize()
    CUR_MASK, CMASK = (1 << 28) - 1, 0xF

    def step(i):
        keys, off = sets[i % nsets]
        if kind == "ralledata":
            from k2hash_amd import ralledata
            (kd, ko, vd, vo), (blob, boff, tot) = keys, off
            ralledata.build_ralledata(kd, ko, vd, vo, out=blob, blob_off=boff, total=tot)
        elif args.index:
            h1, h2 = outs[i % nsets]
            k, c = idx[i % nsets]
            if kind == "fixed":
                batch.hash_fixed_index(keys, shape, CUR_MASK, CMASK, second=args.second, out=(h1, h2, k, c))
            else:
                batch.hash_csr_index(keys, off, CUR_MASK, CMASK, second=args.second, out=(h1, h2, k, c))
        elif kind == "fixed":
            k2hash_amd.hash_fixed(keys, shape, second=args.second, out=outs[i % nsets])
        else:
            k2hash_amd.hash_csr(keys, off, second=args.second, out=outs[i % nsets])

    elapsed, kern_s, extra = timed(step, args.steps, args.warmup, args.warm_ms, world, dist, dev, label="headline")
    total_keys = (total if strong else n * world) * args.steps
    value = total_keys / elapsed

    # --- verification against the reference's digests (outside the timed region) ---------
    verify = None
    if not args.no_verify and strong:
        chunks = golden_chunks(kind, shape, total)
        if chunks:
            verify = verify_sharded(outs[0][0], first, chunks, dist if use_dist else None, dev)
    elif not args.no_verify and kind == "fixed" and not args.keys:
        gname = {"fixed32": "fixed32_16M", "fixed4096": "fixed4096_1M"}[name]
        g = _golden()[gname]
        if name == "fixed32":  # set 0 of rank 0 is exactly the reference's 16M-key workload
            verify = {"ok": rank != 0 or digest_dev(outs[0][0], 0) == g["h1"], "chunks_checked": 1}
        else:
            verify = verify_chunks(outs[0][0], first, g.get("chunks") or [dict(first=0, count=g["n"], h1=g["h1"])])
        if use_dist:
            t = torch.tensor([0 if verify["ok"] else 1, verify["chunks_checked"]], dtype=torch.int64, device=dev)
            dist.all_reduce(t)
            verify = {"ok": int(t[0].item()) == 0, "chunks_checked": int(t[1].item()), "ranks": world}

    # --- the gather of every shard's hashes to rank 0 (RCCL over xGMI) ---------------------
    gather = None
    if use_dist:
        if cuts is not None:
            counts = [b - a for a, b in cuts]
        elif strong:
            counts = shard.shard_counts(total, world)
        else:
            counts = [n] * world
        gsteps = max(3, min(10, args.steps // 10))
        gather, res = measure_gather(outs[0][0], counts, step, gsteps, dist, dev, torch.cuda.synchronize)
        if rank == 0 and not args.no_verify and strong:
            chunks = golden_chunks(kind, shape, total)
            gather["verify_root"] = verify_chunks(res, 0, chunks) if chunks else None
        else:
            gather["verify_root"] = None
        if cuts is not None:
            gather["shard_key_bytes"] = cut_bytes  # the byte cuts: ~equal key bytes per rank
        del res

    secondary = None
    cpu = None
    if rank == 0 and world == 1 and name == "fixed32" and not (args.index or args.second or args.keys):
        if not args.no_secondary:
            del sets, outs
            torch.cuda.empty_cache()
            vf = not args.no_verify
            secondary = {
                "csr": secondary_csr(dev, 20, 60.0, vf, cpu=not args.no_cpu_baseline),
                "fixed4096": secondary_fixed("fixed4096", dev, 20, 60.0, vf, "fixed4096_1M",
                                             cpu=not args.no_cpu_baseline),
                "fixed32_1g": secondary_fixed("fixed32_1g", dev, 10, 60.0, vf, "fixed32_1G"),
                "fixed32_index": secondary_index(dev, 20, 60.0, vf),
                "ralledata": secondary_ralledata(dev, 20, 60.0, vf),
                "import": secondary_import(dev, 10, 60.0, vf),
                "import_mdbm": secondary_import_mdbm(dev, 10, 60.0, vf),
                "host": secondary_host(dev),
            }
            cb = secondary["csr"].get("cpu_baseline")
            if cb:  # the host path's CSR rate beside the reference on the box's cores (same key mix)
                hc = secondary["host"]["csr_8M"]
                hc["cpu_reference_cores"] = {"threads": cb["cores"]["threads"], "value": cb["cores"]["value"],
                                             "key_gb_per_s": cb["cores"]["key_gb_per_s"]}
                hc["host_path_over_cpu_cores"] = hc["value"] / cb["cores"]["value"]
        if not args.no_cpu_baseline:
            host = batch.synth_bytes(n * shape, dev).cpu().numpy()
            cpu = cpu_baseline(host, shape, n)

    if rank == 0:
        model = (n / 64 * chunks_of(shape) * FNV_OPS_PER_CHUNK if kind == "fixed"
                 else key_bytes / 16 * FNV_OPS_PER_CHUNK / 64)
        prof_name = f"{name}{'_index' if args.index else ''}{'_h2' if args.second else ''}"
        line = {
            "metric": METRIC if kind == "fixed" and shape == 32 and not (args.index or args.second)
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
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u64 (u8 key bytes in)",
            "data": "synthetic (splitmix64 counter stream, generated on device; SURVEY.md 8d spec in DESIGN.md)",
            "config": {"workload": desc + (f" -- one batch of {total} keys cut by bytes over {world} ranks"
                                           if cuts is not None else ""),
                       "keys_per_gpu": n, "keys_total": total if strong else n * world,
                       "key_len": shape if kind == "fixed" else list(shape),
                       "second_hash": bool(args.second), "bucket_index": bool(args.index),
                       "parallelism": f"shard{world}"},
            "key_gib_per_s": value * (key_bytes / n) / 2**30,
            "kernel_ms": kern_s * 1e3,
            "roofline": roofline(prof_name, algo_bytes, kern_s, model, n),
            "verify": verify,
            "cpu_baseline": cpu,
        }
        if gather:
            line["gather"] = gather
        if secondary:
            line["secondary"] = secondary
        print(json.dumps(line), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
