#!/bin/bash
# round 3 (session 2): RALLEDATA gather kernel : the piece table built by waves 1-3 during the hash (bisection + forward walk)
# -- RALLEDATA GPU tests, then A/B against the HEAD build
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ralledata.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03aq_pytest_ralle.txt 2>&1
tail -2 gpurun_out/r03aq_pytest_ralle.txt
timeout -k 10 300 python -u tools/ab_libs.py --config ralledata --libs k2hash_amd/lib/ab/HEAD/libk2hash_amd.so --rounds 11 --reps 10 > gpurun_out/r03aq_ralle_ab.txt 2>&1
grep -v amdgpu.ids gpurun_out/r03aq_ralle_ab.txt
echo R03AQ_OK
