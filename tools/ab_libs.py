#!/usr/bin/env python3
"""A/B timing of two builds of the batch library in ONE process (interleaved rounds):
the working tree's k2hash_amd/lib/libk2hash_amd.so against other builds (tools/build_ab.sh).
Every library's output is checked against the golden digest before it is timed.

  python tools/ab_libs.py --libs k2hash_amd/lib/ab/HEAD/libk2hash_amd.so [--config csr] [--variant 0]
"""
import argparse
import ctypes
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from k2hash_amd import _native, batch  # noqa: E402
import oracle  # noqa: E402  (checker only)

p = argparse.ArgumentParser()
p.add_argument("--libs", default="", help="comma list of extra library paths (the tree's own is always first)")
p.add_argument("--config", default="csr")
p.add_argument("--variant", type=int, default=0)
p.add_argument("--rounds", type=int, default=5)
p.add_argument("--reps", type=int, default=10)
p.add_argument("--second", action="store_true")
p.add_argument("--index", action="store_true", help="fixed keys: the fused bucket-index form (kindex + ckindex)")
a = p.parse_args()

dev = torch.device("cuda:0")
if a.config == "ralledata":  # the bench's RALLEDATA workload, checked against its oracle digest
    import bench  # noqa: E402
    _, n, ((klo, khi), (vlo, vhi)), _ = bench.CONFIGS["ralledata"]
    cfg = {"kind": "ralledata"}
    gr = json.loads((ROOT / "tests" / "golden" / "ralledata_digest.json").read_text())
    ko = batch.synth_offsets(n, dev, klo, khi)
    vo = batch.synth_offsets(n, dev, vlo, vhi, seed=batch.SEED_LENS + 7)
    kb, vb = int(ko[-1].item()), int(vo[-1].item())
    kd = batch.synth_bytes(kb, dev)
    vd = batch.synth_bytes(vb, dev, byte_off=1 << 33)
    total = 80 * n + kb + vb
    blob = torch.zeros((total + 7) // 8 * 8, dtype=torch.uint8, device=dev)
    boff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    algo = 2 * (kb + vb) + 104 * n  # input + blob bytes, two offset arrays in, blob offsets out
else:
    dig = json.loads((ROOT / "tests/golden/digests.json").read_text())["configs"]
    name = {"fixed32": "fixed32_16M", "csr": "csr_8_256_64M", "fixed4096": "fixed4096_1M", "fixed21": "fixed21_1M"}[a.config]
    cfg = dig[name]
    n = cfg["n"]
sets = []
for s in range(2 if cfg["kind"] != "ralledata" else 0):
    if cfg["kind"] == "fixed":
        sets.append((batch.synth_bytes(n * cfg["key_len"], dev), None))
        algo = n * cfg["key_len"] + 8 * n
    else:
        off = batch.synth_offsets(n, dev, cfg["min_len"], cfg["max_len"])
        sets.append((batch.synth_bytes(int(off[-1].item()), dev), off))
        algo = int(off[-1].item()) + 16 * n + 8
if a.second:
    algo += 8 * n
if a.index:
    algo += 16 * n
    idx = (torch.empty(n, dtype=torch.int64, device=dev), torch.empty(n, dtype=torch.int64, device=dev))
out = (torch.empty(n, dtype=torch.int64, device=dev), torch.empty(n, dtype=torch.int64, device=dev))

paths = [str(_native.BATCH_LIB)] + [x for x in a.libs.split(",") if x]
libs = []
for path in paths:
    lib = _native._bind(ctypes.CDLL(str(Path(path).resolve())), _native.SIGNATURES.keys())
    if a.variant:
        lib.k2h_amd_set_variant(a.variant)
    libs.append(lib)


def run(lib, i):
    if cfg["kind"] == "ralledata":
        rc = lib.k2h_amd_build_ralledata(kd.data_ptr(), ko.data_ptr(), vd.data_ptr(), vo.data_ptr(), None, None, None,
                                         None, n, blob.data_ptr(), boff.data_ptr(), 0,
                                         torch.cuda.current_stream().cuda_stream)
        assert rc == 0, rc
        return
    keys, off = sets[i & 1]
    h2 = out[1].data_ptr() if a.second else None
    stream = torch.cuda.current_stream().cuda_stream
    if off is None and a.index:
        rc = lib.k2h_amd_hash_fixed_index(keys.data_ptr(), cfg["key_len"], n, out[0].data_ptr(), h2, 0,
                                          (1 << 28) - 1, 0xF, idx[0].data_ptr(), idx[1].data_ptr(), stream)
    elif off is None:
        rc = lib.k2h_amd_hash_fixed(keys.data_ptr(), cfg["key_len"], n, out[0].data_ptr(), h2, 0, stream)
    else:
        rc = lib.k2h_amd_hash_csr(keys.data_ptr(), off.data_ptr(), n, out[0].data_ptr(), h2, 0, stream)
    assert rc == 0, rc


for path, lib in zip(paths, libs):
    if cfg["kind"] == "ralledata":
        blob.zero_()
        boff.zero_()
        run(lib, 0)
        torch.cuda.synchronize()
        ok = gr["n"] == n and gr["bytes"] == total and bench.digest_dev(blob.view(torch.int64), 0) == gr["blob"] \
            and bench.digest_dev(boff, 0) == gr["blob_off"]
        print(f"{path}: parity {'OK' if ok else 'MISMATCH'}", flush=True)
        if not ok:
            sys.exit(1)
        continue
    out[0].zero_()
    run(lib, 0)
    torch.cuda.synchronize()
    ok = [f"{x:016x}" for x in oracle.digest(out[0].cpu().numpy().view(np.uint64))] == cfg["h1"]
    if a.second:
        ok = ok and [f"{x:016x}" for x in oracle.digest(out[1].cpu().numpy().view(np.uint64))] == cfg["h2"]
    print(f"{path}: parity {'OK' if ok else 'MISMATCH'}", flush=True)
    if not ok:
        sys.exit(1)

times = {p_: [] for p_ in paths}
for r in range(a.rounds):
    for path, lib in zip(paths, libs):
        for i in range(3):
            run(lib, i)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(a.reps):
            run(lib, i)
        e1.record()
        torch.cuda.synchronize()
        times[path].append(e0.elapsed_time(e1) / a.reps)
for path in paths:
    med = statistics.median(times[path])
    print(json.dumps({"config": a.config, "lib": path, "variant": a.variant, "ms_median": med,
                      "ms_min": min(times[path]), "frac_8TBps": algo / med / 1e6 / 8000,
                      "Gkeys_s": n / med / 1e6}), flush=True)
