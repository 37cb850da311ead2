#!/bin/bash
# Round 2: GPU test suite, default bench line, and a kernel-trace profile of the headline.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02b_pytest.txt 2>&1
tail -3 gpurun_out/r02b_pytest.txt
timeout -k 10 400 python -u bench.py > gpurun_out/r02b_bench.json 2> gpurun_out/r02b_bench.err
cat gpurun_out/r02b_bench.json
