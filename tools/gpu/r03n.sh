#!/bin/bash
# round 3: import tests with the >4 GiB file
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_import.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03n_pytest_import.txt 2>&1
echo IMPORT_TESTS_OK
echo R03N_OK
