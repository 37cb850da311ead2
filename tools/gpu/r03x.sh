#!/bin/bash
# round 3: import tests + timing after pass B loads the block's speculative list beside the events
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_import.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03x_pytest_import.txt 2>&1
tail -2 gpurun_out/r03x_pytest_import.txt
timeout -k 10 600 bash tools/gpu/r03_import_prof.sh
timeout -k 10 300 python tools/import_step.py --calls 20 > gpurun_out/r03x_import_step.txt 2>&1
tail -1 gpurun_out/r03x_import_step.txt
echo R03X_OK
