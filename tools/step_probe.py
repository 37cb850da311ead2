#!/usr/bin/env python3
"""Cycles per 16-byte FNV step of one wave per SIMD for the walk's loop-body pieces
(tools/lab/src/lab_csr_rs.inc, rs_step_probe_kernel; mode 4 counts each of its two
interleaved chains' steps; modes 7, 8 run two waves per SIMD and report cycles per wave-step
and the wall time per SIMD step, i.e. half a wave-step): s_memtime cycles per step, and the
wall time per step from HIP events (the two give the shader clock)."""
import ctypes
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def main():
    import torch
    lib = ctypes.CDLL(str(ROOT / "tools" / "lab" / "libk2hash_lab.so"))
    lib.k2h_lab_step_probe.restype = ctypes.c_int
    lib.k2h_lab_step_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint, ctypes.c_uint, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    blocks = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    out = torch.zeros(blocks * 8 + blocks * 256, dtype=torch.int64, device=dev)
    sh = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = {}
    for mode in [int(m) for m in sys.argv[3].split(',')] if len(sys.argv) > 3 else (0, 1, 2, 3, 4, 5, 6, 7, 8, 0):
        for _ in range(3):  # warm (clock ramp)
            assert lib.k2h_lab_step_probe(mode, ctypes.c_void_p(out.data_ptr()), blocks, iters, sh) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        assert lib.k2h_lab_step_probe(mode, ctypes.c_void_p(out.data_ptr()), blocks, iters, sh) == 0
        e1.record()
        torch.cuda.synchronize()
        per = 8 if mode == 4 else 4  # chain steps per loop iteration (mode 4: two chains)
        waves = 8 if mode in (7, 8) else 4  # modes 7, 8: two waves per SIMD; wall time per SIMD step
        cyc = out[:blocks * waves].cpu().double() / (per * iters)
        wall_ns = e0.elapsed_time(e1) * 1e6 / (per * iters) / (2 if mode in (7, 8) else 1)
        fin = out[blocks * 8:].cpu()
        res[f"mode{mode}"] = {"final_state_sum": int(fin.sum().item()) & 0xFFFFFFFFFFFF,"cycles_per_step_median": statistics.median(cyc.tolist()),
                              "cycles_per_step_max": cyc.max().item(), "wall_ns_per_step": wall_ns,
                              "clock_ghz_est": statistics.median(cyc.tolist()) / wall_ns}
    print(json.dumps({"blocks": blocks, "iters": iters, "results": res}))


if __name__ == "__main__":
    main()
