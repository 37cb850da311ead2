"""Count the keys the k2himport device scan hashes from the file (pass A named no slot for
them) with a probe library whose miss path stores a marker (tools/probe_build.py, the
'if (code == 0xFFu)' branch replaced by a = c = 0x5EED), for the TSV and mdbm workloads.

    python3 tools/import_miss_probe.py k2hash_amd/lib/probe/p_miss.so
"""
import ctypes
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import bench  # noqa: E402
from k2hash_amd import _native, archive  # noqa: E402


def main():
    _native._batch = _native._bind(ctypes.CDLL(str(Path(sys.argv[1]).resolve())), _native.SIGNATURES.keys())
    dev = torch.device("cuda", 0)
    for fmt in ("tsv", "mdbm"):
        data = bench.import_workload(dev) if fmt == "tsv" else bench.import_mdbm_workload(dev)[0]
        recs, h1, h2 = archive.import_scan_prehash_device(data, fmt)
        miss = int((h1 == 0x5EED).sum().item())
        print(json.dumps({"fmt": fmt, "records": int(recs.shape[0]), "misses": miss,
                          "miss_frac": miss / max(1, recs.shape[0])}), flush=True)
        del data, recs, h1, h2
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
