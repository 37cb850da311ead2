#!/bin/bash
# round 3: import tests and profile after the v_perm span-function compose
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_import.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03l_pytest_import.txt 2>&1
echo IMPORT_TESTS_OK
timeout -k 10 600 bash tools/gpu/r03_import_prof.sh
timeout -k 10 300 python tools/import_step.py --calls 20 > gpurun_out/r03l_import_step.txt 2>&1
tail -3 gpurun_out/r03l_import_step.txt
echo R03L_OK
