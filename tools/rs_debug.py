#!/usr/bin/env python3
"""Lab debug run of a role-split CSR variant on small inputs: compares its hashes with the
product kernel's (variant 0) and prints the lab watchdog record (k2h_lab_r2_dbg) after
each launch.  Usage: python tools/rs_debug.py VARIANT [n ...]"""
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch

    from k2hash_amd import batch
    sys.path.insert(0, str(ROOT / "tools"))
    import lab_ab
    lib = lab_ab.lab_lib()
    lib.k2h_lab_r2_dbg.restype = ctypes.c_int  # (lab_ab.lab_lib binds the csr entry points)
    lib.k2h_lab_r2_dbg.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda:0")
    v = int(sys.argv[1])
    sizes = [int(x) for x in sys.argv[2:]] or [1, 511, 512, 513, 4096, 100000, 1 << 20]
    sh = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    dbg = (ctypes.c_uint32 * 8)()
    for n in sizes:
        off = batch.synth_offsets(n, dev, 8, 256)
        data = batch.synth_bytes(max(int(off[-1].item()), 1), dev)
        ref = torch.zeros(n, dtype=torch.int64, device=dev)
        out = torch.zeros(n, dtype=torch.int64, device=dev)
        assert lib.k2h_lab_csr(0, ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(off.data_ptr()), n,
                               ctypes.c_void_p(ref.data_ptr()), None, sh) == 0
        fn = lib.k2h_lab_csr_lean4 if v >= 53 else lib.k2h_lab_csr_lean if v >= 50 else lib.k2h_lab_csr_rs4 if v >= 40 else lib.k2h_lab_csr_rs2 if v >= 30 else lib.k2h_lab_csr_rs
        assert fn(v, ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(off.data_ptr()), n,
                  ctypes.c_void_p(out.data_ptr()), None, sh) == 0
        torch.cuda.synchronize()
        lib.k2h_lab_r2_dbg(dbg)
        bad = int((ref != out).sum().item())
        print(f"n={n} mismatches={bad} watchdog={list(dbg)}", flush=True)
        if bad:  # which 512-key tiles: index, block (tile % G for G = 2 x CUs), j = tile // G, span
            G = 2 * torch.cuda.get_device_properties(dev).multi_processor_count
            badk = (ref != out).nonzero().flatten().cpu()
            tiles = sorted(set((badk // 512).tolist()))
            offc = off.cpu()
            rows = []
            for t in tiles[:24]:
                k0, k1 = t * 512, min(n, t * 512 + 512)
                nb = int(((badk >= k0) & (badk < k1)).sum())
                rows.append((t, t % G, t // G, nb, int(offc[k1] - offc[k0])))
            print(f"  bad tiles={len(tiles)} (tile, block, j, bad keys, span): {rows}", flush=True)
            k0 = int(tiles[0]) * 512
            kb = [int(k) for k in badk if k < k0 + 512]
            lens = [int(offc[k + 1] - offc[k]) for k in kb]
            refc, outc = ref.cpu(), out.cpu()
            zero = sum(int(outc[k] == 0) for k in kb)
            other = sum(int((refc[k0:k0 + 512] == outc[k]).any()) for k in kb)
            print(f"  tile {tiles[0]}: keys {[k - k0 for k in kb]} lens {lens} out==0: {zero} "
                  f"out==another key's hash: {other}", flush=True)
            js = [t // G for t in tiles]
            print(f"  by j: {[js.count(j) for j in range(max(js) + 1)]}", flush=True)


if __name__ == "__main__":
    main()
