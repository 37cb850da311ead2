#!/bin/bash
# round 3: TSV import with the in-kernel entry-state scan and the split speculative list:
# import tests, then the import profile (trace + PMC passes)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_import.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03j_pytest_import.txt 2>&1
echo IMPORT_TESTS_OK
timeout -k 10 600 bash tools/gpu/r03_import_prof.sh

timeout -k 10 500 python -u bench.py > gpurun_out/r03j_bench.json 2> gpurun_out/r03j_bench.err
echo BENCH_OK
echo R03J_OK
