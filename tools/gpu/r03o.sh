#!/bin/bash
# round 3: bench tests on the GPU, including the RCCL one-rank rehearsal of the N>1 path
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_bench.py -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r03o_pytest_bench.txt 2>&1 || { tail -40 gpurun_out/r03o_pytest_bench.txt; exit 1; }
tail -5 gpurun_out/r03o_pytest_bench.txt
echo R03O_OK
