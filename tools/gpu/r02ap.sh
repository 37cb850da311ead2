#!/bin/bash
# TSV device scan (compact functions): import GPU tests, rate, kernel times
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/imp_prof7
timeout -k 10 300 python -u -m pytest tests/test_import.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/imp_tests.txt 2>&1
tail -3 gpurun_out/imp_tests.txt
timeout -k 10 200 python -u tools/import_rate.py > gpurun_out/import_rate.json
cat gpurun_out/import_rate.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/imp_prof7 -o run -- python3 -u tools/import_rate.py --reps 3 > gpurun_out/imp_prof7/rate.json 2> gpurun_out/imp_prof7/err.txt
