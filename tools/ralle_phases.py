#!/usr/bin/env python3
"""Per-block phase times of the RALLEDATA gather kernel (lab variant 76: shader-clock
stamps by thread 0 at entry, after the staging barrier, after the hash barrier, and after
its output pieces).  Prints medians / means in cycles and in us at the clock_probe clock,
and the mean number of resident blocks implied by block lifetime x blocks / kernel time.

  python tools/ralle_phases.py [--clock-ghz 2.1]
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

from k2hash_amd import _native, batch, ralledata  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--clock-ghz", type=float, default=2.1)
p.add_argument("--n", type=int, default=1 << 23)
p.add_argument("--variant", type=int, default=76, help="76: stamps, 77: stamps without the piece stores")
a = p.parse_args()
dev = torch.device("cuda:0")
n = a.n
ko = batch.synth_offsets(n, dev, 8, 64)
vo = batch.synth_offsets(n, dev, 0, 256, seed=batch.SEED_LENS + 7)
kb, vb = int(ko[-1].item()), int(vo[-1].item())
kd, vd = batch.synth_bytes(kb, dev), batch.synth_bytes(vb, dev, byte_off=1 << 33)
blob = torch.empty(80 * n + kb + vb, dtype=torch.uint8, device=dev)
boff = torch.empty(n + 1, dtype=torch.int64, device=dev)


def run():
    ralledata.build_ralledata(kd, ko, vd, vo, out=blob, blob_off=boff, total=blob.numel())


_native.lab_set_variant(0)
for _ in range(200):
    run()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
_native.lab_set_variant(a.variant)
run()
e0.record()
run()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1)
nb = n // 64
st = boff[:nb * 64].view(nb, 64)[:, :6].double()
ph = {"span offsets": st[:, 4] - st[:, 0], "records (wave 0)": st[:, 5] - st[:, 4], "stage wait + barrier": st[:, 1] - st[:, 5],
      "hash": st[:, 2] - st[:, 1], "pieces(wave0)": st[:, 3] - st[:, 2], "life(wave0)": st[:, 3] - st[:, 0]}
res = {"kernel_ms": ms, "blocks": nb}
for k, v in ph.items():
    res[k] = {"median_cyc": v.median().item(), "mean_cyc": v.mean().item(),
              "p90_cyc": v.quantile(0.9).item() if v.numel() < 16_000_000 else None,
              "mean_us": v.mean().item() / a.clock_ghz / 1e3}
res["resident_blocks_mean"] = nb * res["life(wave0)"]["mean_us"] / (ms * 1e3)
print(json.dumps(res, indent=1))
