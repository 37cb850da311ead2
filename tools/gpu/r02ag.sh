#!/bin/bash
# TSV device scan as the getline machine: import GPU tests, then the rate tool
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_import.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/imp_tests.txt 2>&1
tail -3 gpurun_out/imp_tests.txt
timeout -k 10 200 python -u tools/import_rate.py > gpurun_out/import_rate.json
cat gpurun_out/import_rate.json
