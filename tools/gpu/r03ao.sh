#!/bin/bash
# round 3 (session 2): import record count returned through mapped pinned host memory (no read-back copy command)
# -- import
# GPU tests, then same-process A/B against the HEAD build
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_import.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ao_pytest_import.txt 2>&1
tail -2 gpurun_out/r03ao_pytest_import.txt
timeout -k 10 300 python -u tools/import_step.py --ab k2hash_amd/lib/ab/HEAD/libk2hash_amd.so --calls 10 --rounds 9 > gpurun_out/r03ao_import_ab.txt 2>&1
grep -v amdgpu.ids gpurun_out/r03ao_import_ab.txt
echo R03AO_OK
