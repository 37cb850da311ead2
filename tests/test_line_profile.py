"""The line-profile tooling: bench.py's roctx ranges are off unless asked
for, and tools/summarize_line_profile.py recomputes each entry's fraction from the kernels
inside its range (synthetic rocprofv3 CSVs here; the GPU run is tools/profile_line.sh)."""
import json
import subprocess
import sys

from conftest import ROOT


def test_bench_markers_off_by_default(monkeypatch):
    sys.path.insert(0, str(ROOT))
    import bench

    monkeypatch.delenv("K2H_BENCH_MARKERS", raising=False)
    bench._ROCTX.clear()
    assert bench._roctx() is None
    bench._ROCTX.clear()


def _write(tmp_path, line, kernels, ranges):
    (tmp_path / "bench_line.json").write_text(json.dumps(line) + "\n")
    tr = tmp_path / "trace"
    tr.mkdir()
    (tr / "run_kernel_trace.csv").write_text(
        "Kernel_Name,Start_Timestamp,End_Timestamp\n" + "".join(f'"{n}",{a},{b}\n' for n, a, b in kernels))
    (tr / "run_marker_api_trace.csv").write_text(
        '"Domain","Function","Process_Id","Thread_Id","Correlation_Id","Start_Timestamp","End_Timestamp"\n'
        + "".join(f'"MARKER_CORE_RANGE_API","timed:{lab}",1,1,{i},{a},{b}\n' for i, (lab, a, b) in enumerate(ranges)))


def test_summarize_line_profile_recomputes_each_entry(tmp_path):
    algo = 8_000_000  # bytes per launch: 8e6 / 1e-6 s = 8 TB/s at a 1 us window
    line = {"steps": 3, "ms_per_step": 0.002, "kernel_ms": 0.002, "roofline": {"frac": 0.5, "algorithmic_bytes_per_launch": algo},
            "secondary": {"csr": {"steps": 2, "ms_per_step": 0.001, "kernel_ms": 0.001,
                                  "roofline": {"frac": 1.0, "algorithmic_bytes_per_launch": algo}},
                          "import": {"steps": 2, "ms_per_step": 0.004,
                                     "roofline": {"frac": 0.25, "algorithmic_bytes_per_launch": algo}}}}
    k = []
    # headline range [0, 10000): three 2-us dispatches of the dominant kernel + a synth kernel
    k += [("fnv_fixed32_kpt_kernel", 1000 + 3000 * i, 3000 + 3000 * i) for i in range(3)]
    k += [("synth_bytes_kernel", 100, 900), ("fnv_fixed32_kpt_kernel", 20000, 30000)]  # outside: ignored
    # csr range [40000, 50000): two 1-us dispatches + a short other kernel
    k += [("fnv_csr_staged_kernel", 41000, 42000), ("fnv_csr_staged_kernel", 43000, 44000), ("other", 45000, 45100)]
    # import range [60000, 68000): two calls of three kernels
    k += [("tsv_a_kernel", 60500, 62000), ("tsv_scan_kernel", 62100, 62300), ("tsv_b_kernel", 62400, 63500)]
    k += [("tsv_a_kernel", 64500, 66000), ("tsv_scan_kernel", 66100, 66300), ("tsv_b_kernel", 66400, 67500)]
    _write(tmp_path, line, k, [("headline", 0, 10000), ("csr", 40000, 50000), ("import", 60000, 68000)])
    out = tmp_path / "summary.json"
    subprocess.run([sys.executable, str(ROOT / "tools" / "summarize_line_profile.py"), str(tmp_path), "t", str(out)],
                   check=True, capture_output=True)
    e = json.loads(out.read_text())["entries"]
    assert e["headline"]["dominant"] == "fnv_fixed32_kpt_kernel" and e["headline"]["dispatches_ok"]
    assert abs(e["headline"]["window_us"] - 2.0) < 1e-9 and abs(e["headline"]["frac_profile"] - 0.5) < 1e-9
    assert abs(e["csr"]["frac_profile_over_line"] - 1.0) < 1e-9
    # whole calls: the range's span / steps (8 us / 2 = 4 us per call)
    assert abs(e["import"]["window_us"] - 4.0) < 1e-9 and abs(e["import"]["frac_profile"] - 0.25) < 1e-9
    assert abs(e["import"]["kernel_sum_per_call_us"] - 2.8) < 1e-9
