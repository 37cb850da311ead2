#!/bin/bash
# Round 3 final: GPU suite, default bench line, import profile (after the pinned-count change)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r03ap_pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/r03ap_pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/r03ap_pytest_gpu.txt
timeout -k 10 400 python bench.py > gpurun_out/r03ap_bench.json 2> gpurun_out/r03ap_bench.err || { tail -20 gpurun_out/r03ap_bench.err; exit 1; }
timeout -k 10 600 bash tools/gpu/r03_import_prof.sh || exit 1
echo R03AP_OK
