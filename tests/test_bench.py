"""bench.py's launcher and multi-rank path.

The driver runs `python bench.py --gpus N` (or the same under torch.distributed.run); with
no RANK / WORLD_SIZE in the environment bench.py starts its own N ranks before touching a
GPU.  On CPU the plumbing is rehearsed with the scalar plugin over gloo; on the GPU box two
ranks share cuda:0 (gloo, device tensors staged through host memory) and run the real
kernels, the digest checks and the gather."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _run(args, timeout):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    p = subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_launcher_rehearsal_cpu():
    line = _run(["--gpus", "2", "--rehearse-cpu", "--backend", "gloo", "--steps", "2", "--warmup", "1",
                 "--keys", "777"], 240)
    assert line["n_gpus"] == 2 and line["gather"]["ok"] is True
    assert "NOT a measurement" in line["device"]


def test_launcher_rehearsal_cpu_three_ranks():
    line = _run(["--gpus", "3", "--rehearse-cpu", "--backend", "gloo", "--steps", "1", "--warmup", "0",
                 "--keys", "1001"], 240)
    assert line["n_gpus"] == 3 and line["gather"]["ok"] is True


def _torchrun(nproc, args, timeout):
    """The driver's N > 1 command form: python -m torch.distributed.run --nnodes=1
    --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N ..."""
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
                        "--master-addr", "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"),
                        "--gpus", str(nproc)] + args, capture_output=True, text=True, timeout=timeout, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("config", ["fixed32_1g", "csr"])
def test_rehearsal_eight_ranks_driver_command_form(config):
    """the full N = 8 command form the driver uses, rehearsed on CPU (gloo,
    scalar plugin): eight ranks, the per-rank counts, bytes_to_root, seven point-to-point
    receives at the root, the sharded digest check and the gathered vector; for csr one
    batch cut by bytes (shard_key_bytes balanced, counts uneven)."""
    total = 4000
    line = _torchrun(8, ["--rehearse-cpu", "--config", config, "--steps", "1", "--warmup", "0",
                         "--keys", str(total)], 300)
    g = line["gather"]
    assert line["n_gpus"] == 8 and line["scaling"] == "strong" and line["config"]["keys_total"] == total
    assert len(g["counts"]) == 8 and sum(g["counts"]) == total and g["p2p_peers_at_root"] == 7
    assert g["bytes_to_root"] == 8 * (total - g["counts"][0])
    assert g["ok"] is True and g["verify_root"]["ok"] is True
    assert line["verify"]["ok"] is True and line["verify"]["ranks"] == 8
    if config == "csr":
        kb = g["shard_key_bytes"]
        assert len(kb) == 8 and max(kb) - min(kb) <= 2 * 256


def test_launcher_fails_fast_when_a_rank_dies():
    """A rank that dies after joining the process group (--inject-rank-failure, test only)
    must end the whole run with a non-zero status well inside the driver's limit, with no
    rank left running (rank 0 would otherwise block in its first collective)."""
    import time

    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "3", "--rehearse-cpu", "--backend", "gloo",
                        "--steps", "1", "--warmup", "0", "--keys", "99", "--inject-rank-failure", "1",
                        "--init-timeout", "300"], capture_output=True, text=True, timeout=120, env=env)
    took = time.monotonic() - t0
    assert p.returncode != 0 and took < 60, (p.returncode, took, p.stderr[-2000:])
    assert "rank 1 exited with 3" in p.stderr
    pids = [int(x) for x in p.stderr.split("rank pids [", 1)[1].split("]", 1)[0].split(",")]
    time.sleep(0.5)
    for pid in pids:
        try:
            os.kill(pid, 0)
            alive = Path(f"/proc/{pid}/status").read_text().split("State:")[1].split()[0] != "Z"
        except (ProcessLookupError, FileNotFoundError, IndexError):
            alive = False
        assert not alive, f"rank process {pid} survived the launcher"


def test_roofline_fields_scale_with_keys_per_launch():
    """roofline.traffic / valu_frac come from profiles taken at one key count; a launch of
    another size (config 4 at N = 8: 2^27 keys per rank) must be scaled, not copied."""
    sys.path.insert(0, str(ROOT))
    import bench

    n = 1 << 27
    algo = 40 * n
    r = bench.roofline("fixed32_1g", algo, 0.94e-3, 0.0, n)
    assert r["traffic"] is not None and 0.99 < r["traffic"] / algo < 1.05
    assert 0.3 < r["valu_frac"] < 1.0
    full = bench.roofline("fixed32_1g", 40 << 30, 7.4e-3, 0.0, 1 << 30)
    assert abs(full["valu_insts_per_launch"] / r["valu_insts_per_launch"] - 8.0) < 1e-9
    assert bench.roofline("fixed32_1g", algo, 1e-3, 123.0, None)["traffic"] is None


@pytest.mark.gpu
def test_bench_two_ranks_one_gpu():
    """Config 4's path at N=2 on one card: strong-scaled shards of a small key count, the
    gather of both shards' hashes and the hash+gather step."""
    line = _run(["--gpus", "2", "--backend", "gloo", "--keys", "262144", "--steps", "5", "--warmup", "1",
                 "--warm-ms", "5"], 600)
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["gather"]["with_gather"]["value"] > 0 and line["gather"]["backend"] == "gloo"
    # profile-derived fields are scaled to this launch's key count
    rf = line["roofline"]
    assert rf["keys_per_launch"] == 131072  # --keys is the whole sharded batch
    assert 0 < rf["valu_frac"] < 1.2
    assert rf["traffic"] is None or rf["traffic"] / rf["algorithmic_bytes_per_launch"] < 1.2


@pytest.mark.gpu
def test_bench_rccl_path_one_rank():
    """The driver's N>1 command form (torch.distributed.run, one process per GPU) at one
    rank with --dist: RCCL (backend nccl) initialised with device_id and a timeout, the
    barrier-bracketed timing with its MAX all-reduce on a device tensor, and the gather, on
    the one GPU this box has (two ranks cannot share a GPU under RCCL).  The 8-GPU run
    itself is the driver's."""
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"),
                        "--gpus", "1", "--dist", "--config", "fixed32_1g", "--keys", "262144", "--steps", "5",
                        "--warmup", "1", "--warm-ms", "5"], capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["scaling"] == "strong"
    assert line["gather"]["backend"] == "nccl" and line["gather"]["with_gather"]["value"] > 0


@pytest.mark.gpu
def test_bench_n1_headline_verified():
    line = _run(["--steps", "5", "--warmup", "2", "--warm-ms", "10", "--no-secondary", "--no-cpu-baseline"], 600)
    assert line["n_gpus"] == 1 and line["verify"]["ok"] is True
    assert 0 < line["roofline"]["frac"] < 1 and 0 < line["roofline"]["valu_frac"] < 1.2


def test_digest_and_chunk_check_match_oracle(oracle):
    """bench.py's on-device verification (digest_dev / verify_chunks), run on CPU tensors:
    equal to the oracle's digest, including a chunk that starts at a non-zero global key
    index, and a chunk outside the shard is skipped, a corrupted one fails."""
    import numpy as np
    import torch

    sys.path.insert(0, str(ROOT))
    import bench

    h = np.random.default_rng(5).integers(0, 2**63, size=10007, dtype=np.int64).view(np.uint64)
    t = torch.from_numpy(h.view(np.int64).copy())
    assert bench.digest_dev(t, 0) == [f"{x:016x}" for x in oracle.digest(h)]
    first = 3000
    chunks = [dict(first=3000, count=5000, h1=[f"{x:016x}" for x in oracle.digest(h[3000:8000], 3000)]),
              dict(first=0, count=100, h1=["0"] * 3)]  # outside [first, first + n): skipped
    r = bench.verify_chunks(t[first:], first, chunks)
    assert r == {"chunks_checked": 1, "ok": True}
    bad = t[first:].clone()
    bad[17] ^= 1
    assert bench.verify_chunks(bad, first, chunks)["ok"] is False


def test_bench_measures_the_baseline_metric_and_configs():
    """bench.py's metric string and workloads are BASELINE.json's: config 2 = 16M x 32 B,
    3 = 64M CSR keys of 8-256 B, 4 = 2^30 x 32 B over the GPUs, 5 = 4 KiB keys (1M)."""
    sys.path.insert(0, str(ROOT))
    import bench

    base = json.loads((ROOT / "BASELINE.json").read_text())
    assert bench.METRIC == base["metric"]
    assert bench.CONFIGS["fixed32"][1:3] == (1 << 24, 32) and "16M fixed-length 32B" in base["configs"][1]
    assert bench.CONFIGS["csr"][1:3] == (1 << 26, (8, 256)) and "64M mixed-length keys 8" in base["configs"][2]
    assert bench.CONFIGS["fixed32_1g"][1] is None and bench.KEYS_1G == 1 << 30 and "1B 32B keys" in base["configs"][3]
    assert bench.CONFIGS["fixed4096"][1:3] == (1 << 20, 4096) and "4 KiB keys" in base["configs"][4]


def test_cpu_baseline_workload_csr_and_fixed(oracle):
    """The secondary configs' CPU legs (the reference's scalar hash over the
    exact C3 / C5 inputs) on a small prefix: digests agree with the oracle's hashes."""
    import numpy as np

    sys.path.insert(0, str(ROOT))
    import bench

    off = oracle.gen_offsets(3000, 8, 256)
    data = oracle.gen_bytes(int(off[-1]))
    h1, _ = oracle.hash_csr(data, off)
    r = bench.cpu_baseline_workload("csr", data, off.astype(np.uint64), 0, 500, 3000, h1.copy())
    assert r["digest_matches_gpu"] is True and r["cores"]["keys"] == 3000 and r["single_thread"]["value"] > 0
    keys = oracle.gen_bytes(4096 * 64)
    f1, _ = oracle.hash_fixed(keys, 4096)
    r = bench.cpu_baseline_workload("fixed", keys, None, 4096, 8, 64, f1.copy())
    assert r["digest_matches_gpu"] is True and r["cores"]["key_bytes"] == 64 * 4096
    bad = f1.copy()
    bad[3] ^= 1
    assert bench.cpu_baseline_workload("fixed", keys, None, 4096, 8, 64, bad)["digest_matches_gpu"] is False


def test_cpu_baseline_cores_is_the_process_share(oracle):
    """the headline cpu_baseline is labelled by what this process may use
    (affinity, cgroup quota, OMP_NUM_THREADS), and its value is that pass's; the pass over
    every listed CPU stays a sub-field."""
    sys.path.insert(0, str(ROOT))
    import bench

    keys = oracle.gen_bytes(32 * 20000)
    r = bench.cpu_baseline(keys, 32, 20000)
    cores = bench.usable_cores(bench.host_info())
    assert r["cores"] == cores == r["cpu_share"]["threads"]
    assert r["value"] == r["cpu_share"]["value"]
    assert r["all_listed_cpus"]["threads"] == (os.cpu_count() or cores)


@pytest.mark.gpu
def test_bench_csr_two_ranks_one_batch_cut_by_bytes():
    """bench.py --config csr at N = 2 (two ranks sharing cuda:0 over gloo)
    strong-scales ONE config-3-shaped batch cut by bytes: the reference's 64K-key CSR
    workload (tests/golden/digests.json csr_8_256_64K), each rank hashing its rebased shard
    with the HIP kernel; the per-rank partial digests combine to the reference's and the
    gathered vector at rank 0 matches it too."""
    line = _run(["--gpus", "2", "--backend", "gloo", "--config", "csr", "--keys", "65536", "--steps", "5",
                 "--warmup", "1", "--warm-ms", "5"], 600)
    g = line["gather"]
    assert line["n_gpus"] == 2 and line["scaling"] == "strong" and line["config"]["keys_total"] == 65536
    assert line["verify"]["ok"] is True and line["verify"]["chunks_checked"] == 1
    assert g["verify_root"]["ok"] is True and sum(g["counts"]) == 65536
    kb = g["shard_key_bytes"]
    assert abs(kb[0] - kb[1]) <= 2 * 256


@pytest.mark.gpu
def test_bench_csr_rccl_one_rank():
    """The driver's command form with RCCL at one rank for the CSR strong path (--dist)."""
    line = _torchrun(1, ["--dist", "--config", "csr", "--keys", "65536", "--steps", "5", "--warmup", "1",
                         "--warm-ms", "5"], 600)
    assert line["gather"]["backend"] == "nccl" and line["verify"]["ok"] is True
    assert line["gather"]["verify_root"]["ok"] is True
