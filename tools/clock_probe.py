#!/usr/bin/env python3
"""Shader clock the chip sustains inside the hot kernels (lab clock-probe variants).

Variants 71 / 72 of the lab library run the product fixed32 and 4 KiB-line kernels
unchanged except that every wave stamps s_memtime (shader clock) and s_memrealtime
(100 MHz constant counter) at its start and end into the h2 buffer.  The ratio of the
summed deltas is the clock the waves actually ran at, which turns SQ_INSTS_VALU into a
VALU-utilisation figure without the GRBM_GUI_ACTIVE estimate (unreliable on this box).

  python tools/clock_probe.py [--warm 200] [--json profiles/clock_probe.json]
"""
import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
os.environ.setdefault("K2H_AMD_BATCH_LIB", str(ROOT / "tools" / "lab" / "libk2hash_amd_lab.so"))

import torch  # noqa: E402

import k2hash_amd  # noqa: E402
from k2hash_amd import _native, batch  # noqa: E402

CASES = {"fixed32": (32, 1 << 24, 71), "fixed4096": (4096, 1 << 20, 72), "csr": (None, 1 << 26, 78)}

p = argparse.ArgumentParser()
p.add_argument("--warm", type=int, default=200, help="product launches before the probe (clock ramp)")
p.add_argument("--reps", type=int, default=5)
p.add_argument("--json", default="")
a = p.parse_args()
dev = torch.device("cuda:0")
res = {}
for name, (L, n, var) in CASES.items():
    if L is None:  # BASELINE config 3: CSR keys of 8-256 B
        off = batch.synth_offsets(n, dev, 8, 256)
        keys = batch.synth_bytes(int(off[-1].item()), dev)
        hash_ = lambda out: k2hash_amd.hash_csr(keys, off, out=out)  # noqa: E731
    else:
        keys = batch.synth_bytes(n * L, dev)
        hash_ = lambda out: k2hash_amd.hash_fixed(keys, L, out=out)  # noqa: E731
    h1 = torch.empty(n, dtype=torch.int64, device=dev)
    _native.lab_set_variant(0)
    ref, _ = hash_(None)
    for _ in range(a.warm):
        hash_((h1, None))
    _native.lab_set_variant(var)
    rows = []
    for _ in range(a.reps):
        st = torch.zeros(n, dtype=torch.int64, device=dev)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        hash_((h1, st))
        ev1.record()
        torch.cuda.synchronize()
        s = st.view(-1, 4)
        s = s[s[:, 2] != 0].cpu().double()
        dclk = (s[:, 1] - s[:, 0]).sum().item()
        drt = (s[:, 3] - s[:, 2]).sum().item()
        span_us = (s[:, 3].max() - s[:, 2].min()).item() / 100.0
        rows.append({"waves": int(s.shape[0]), "clock_ghz": round(0.1 * dclk / drt, 4),
                     "wave_us_mean": round(drt / s.shape[0] / 100.0, 3),
                     "span_us": round(span_us, 2), "event_us": round(ev0.elapsed_time(ev1) * 1e3, 2)})
    _native.lab_set_variant(0)
    ok = torch.equal(h1, ref)
    del keys
    res[name] = {"hashes_match": ok, "reps": rows,
                 "clock_ghz": round(sum(r["clock_ghz"] for r in rows[1:]) / max(1, len(rows) - 1), 4)}
    print(name, json.dumps(res[name]), flush=True)
if a.json:
    Path(a.json).write_text(json.dumps(res, indent=1) + "\n")
