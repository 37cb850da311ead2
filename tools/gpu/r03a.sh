#!/bin/bash
# Round 3, first GPU session: the GPU suite on the cleaned product tree (one-launch CSR
# kernel), the default bench line, and a kernel-trace profile of the CSR config.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r03a_pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/r03a_pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/r03a_pytest_gpu.txt
timeout -k 10 300 python bench.py > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err || { tail -20 gpurun_out/r03a_bench.err; exit 1; }
OUT=gpurun_out/prof_r03a bash tools/profile_round.sh csr || exit 1
echo R03A_OK
