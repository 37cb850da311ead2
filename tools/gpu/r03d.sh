#!/bin/bash
# Round 3: single-read TSV import scan (GPU tests, per-call time, rocprof trace + PMC);
# CSR register-staged lab A/B after the store-base fix.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_import.py tests/test_archive.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r03d_pytest.txt 2>&1 || { tail -30 gpurun_out/r03d_pytest.txt; exit 1; }
tail -2 gpurun_out/r03d_pytest.txt
timeout -k 10 120 python tools/import_step.py --calls 20 > gpurun_out/r03d_import_step.txt 2>&1 || { tail gpurun_out/r03d_import_step.txt; exit 1; }
cat gpurun_out/r03d_import_step.txt
timeout -k 10 600 bash tools/gpu/r02ar.sh || exit 1
timeout -k 10 240 python tools/lab_ab.py csr --variants 0 1 --reps 7 > gpurun_out/r03d_csr_ab.json 2> gpurun_out/r03d_csr_ab.err || { tail -20 gpurun_out/r03d_csr_ab.err; exit 1; }
cat gpurun_out/r03d_csr_ab.json
echo R03D_OK
