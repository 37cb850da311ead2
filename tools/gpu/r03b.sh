#!/bin/bash
# Round 3: table-state bucket index GPU tests; 4 KiB persistent line-DMA A/B (lab).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bucket_index.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r03b_pytest.txt 2>&1 || { tail -30 gpurun_out/r03b_pytest.txt; exit 1; }
tail -2 gpurun_out/r03b_pytest.txt
timeout -k 10 240 python tools/lab_ab.py lines --variants 0:0 1:8 1:10 1:4 1:6 > gpurun_out/r03b_lines_ab.json 2> gpurun_out/r03b_lines_ab.err || { tail -20 gpurun_out/r03b_lines_ab.err; exit 1; }
timeout -k 10 240 python tools/lab_ab.py csr --variants 0 1 > gpurun_out/r03b_csr_ab.json 2> gpurun_out/r03b_csr_ab.err || { tail -20 gpurun_out/r03b_csr_ab.err; exit 1; }
cat gpurun_out/r03b_csr_ab.json
cat gpurun_out/r03b_lines_ab.json
echo R03B_OK
