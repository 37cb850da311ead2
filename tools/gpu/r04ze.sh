#!/bin/bash
# Round 4: the new staged/direct pass-B units test, and the import test file
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ze
timeout -k 10 600 python -u -m pytest tests/test_import.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04ze/pytest.txt 2>&1 || { tail -40 gpurun_out/r04ze/pytest.txt; exit 1; }
tail -3 gpurun_out/r04ze/pytest.txt
echo R04ZE_OK
