"""Histogram of why the mdbm device scan's keys miss pass A's slots, from a probe library
whose miss path stores a marker in h1 and a diagnostic word in h2 (slot index js, the slot's
length sj, the key's length, event index j, the head byte, the span's slot events, its event
count, the event offset, over).  Timing-free; run on a GPU box:
    python3 tools/import_miss_diag.py k2hash_amd/lib/probe/p_diag.so
"""
import collections
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
    data = bench.import_mdbm_workload(dev)[0]
    recs, h1, h2 = archive.import_scan_prehash_device(data, "mdbm")
    m = h1 == 0x5EED
    d = h2[m].cpu().numpy().astype("uint64")
    print(json.dumps({"records": int(recs.shape[0]), "misses": int(m.sum().item())}))
    c = collections.Counter()
    for w in d[:200000]:
        w = int(w)
        js, sj, ln, j, hb = w & 3, (w >> 2) & 0xFF, (w >> 10) & 0xFF, (w >> 18) & 63, (w >> 24) & 0xFF
        msi, ne, o, over = (w >> 32) & 0x1FF, (w >> 41) & 7, (w >> 44) & 127, (w >> 51) & 1
        why = ("over" if over else "no-slot(js=3)" if js == 3 else "slot-unnamed(sj=FF)" if sj == 0xFF
               else "len-mismatch")
        c[(why, "j=%d" % min(j, 6), "ne=%d" % ne, "js=%d" % js, "hc=%d" % ((msi & 7) == 0), "head=%s" % (hb != 0xFF))] += 1
    for k, v in c.most_common(25):
        print(v, k)
    ex = [int(w) for w in d[:5]]
    print("examples", [hex(x) for x in ex])


if __name__ == "__main__":
    main()
