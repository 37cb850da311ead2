#!/bin/bash
# round 3 (session 2): the one-statement two-key form for the h2 and fused-index variants
# of fixed32 -- GPU suite, then A/B against HEAD (config 2 with h2; with the fused index)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ag_pytest_gpu.txt 2>&1
tail -2 gpurun_out/r03ag_pytest_gpu.txt
timeout -k 10 300 python -u tools/ab_libs.py --config fixed32 --second --libs k2hash_amd/lib/ab/HEAD/libk2hash_amd.so --rounds 11 --reps 20 > gpurun_out/r03ag_fixed32_ab.txt 2>&1
timeout -k 10 300 python -u tools/ab_libs.py --config fixed32 --index --libs k2hash_amd/lib/ab/HEAD/libk2hash_amd.so --rounds 11 --reps 20 >> gpurun_out/r03ag_fixed32_ab.txt 2>&1
timeout -k 10 300 python -u tools/ab_libs.py --config fixed32 --libs k2hash_amd/lib/ab/HEAD/libk2hash_amd.so --rounds 11 --reps 20 >> gpurun_out/r03ag_fixed32_ab.txt 2>&1
grep -v amdgpu.ids gpurun_out/r03ag_fixed32_ab.txt
echo R03AG_OK
