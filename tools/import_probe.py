"""Probe: kernel times of the k2himport TSV device scan with and without the fused
prehash (tsv_b_kernel<true> vs <false>) on bench's 8M-record workload, under rocprofv3
--kernel-trace (the caller reads the trace).  Calls alternate: scan_prehash, scan only."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import bench  # noqa: E402
from k2hash_amd import _native, archive  # noqa: E402

if len(sys.argv) > 1:  # another build of the library (tools/probe_build.py, build_ab.sh)
    import ctypes
    _native._batch = _native._bind(ctypes.CDLL(str(Path(sys.argv[1]).resolve())), _native.SIGNATURES.keys())
dev = torch.device("cuda", 0)
data = bench.import_workload(dev)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.2:
    archive.import_scan_prehash_device(data)
for _ in range(10):
    archive.import_scan_prehash_device(data)
    archive.import_scan_device(data)
torch.cuda.synchronize()
print("done")
