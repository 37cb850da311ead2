#!/bin/bash
# round 3: the GPU suite and the bench line after the CSR offset-load batching
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r03t_pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/r03t_pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/r03t_pytest_gpu.txt
timeout -k 10 400 python bench.py > gpurun_out/r03t_bench.json 2> gpurun_out/r03t_bench.err || { tail -20 gpurun_out/r03t_bench.err; exit 1; }
OUT=gpurun_out/prof_r03t bash tools/profile_round.sh csr || exit 1
echo R03T_OK
