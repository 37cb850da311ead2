#!/bin/bash
# round 3: import tests after the register-held tile scan; RALLEDATA lab A/B (variants 0, 1, 2)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_import.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03k_pytest_import.txt 2>&1
echo IMPORT_TESTS_OK
timeout -k 10 240 python tools/lab_ab.py ralle --variants 0 1 2 --reps 7 > gpurun_out/r03k_ralle_ab.json 2> gpurun_out/r03k_ralle_ab.err
cat gpurun_out/r03k_ralle_ab.json
timeout -k 10 300 python tools/import_step.py --calls 20 > gpurun_out/r03k_import_step.txt 2>&1
tail -3 gpurun_out/r03k_import_step.txt
echo R03K_OK
