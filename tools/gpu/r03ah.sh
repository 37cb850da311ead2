#!/bin/bash
# round 3 (session 2): RALLEDATA gather kernel : LDS-only barriers, global staged loads, blob offsets written by wave 1 after the first barrier
# -- RALLEDATA GPU tests, then A/B against the HEAD build
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ralledata.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ah_pytest_ralle.txt 2>&1
tail -2 gpurun_out/r03ah_pytest_ralle.txt
timeout -k 10 300 python -u tools/ab_libs.py --config ralledata --libs k2hash_amd/lib/ab/HEAD/libk2hash_amd.so --rounds 11 --reps 10 > gpurun_out/r03ah_ralle_ab.txt 2>&1
grep -v amdgpu.ids gpurun_out/r03ah_ralle_ab.txt
echo R03AH_OK
