#!/bin/bash
# round 3 (session 2): fixed32 two keys per lane as one asm statement (key 0 hashed after
# its own two loads, key 1 in place) -- GPU suite, then A/B against HEAD on config 2
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03af_pytest_gpu.txt 2>&1
tail -2 gpurun_out/r03af_pytest_gpu.txt
timeout -k 10 300 python -u tools/ab_libs.py --config fixed32 --libs k2hash_amd/lib/ab/HEAD/libk2hash_amd.so --rounds 15 --reps 20 > gpurun_out/r03af_fixed32_ab.txt 2>&1
timeout -k 10 300 python -u tools/ab_libs.py --config fixed32 --libs k2hash_amd/lib/ab/HEAD/libk2hash_amd.so --rounds 15 --reps 20 >> gpurun_out/r03af_fixed32_ab.txt 2>&1
grep -v amdgpu.ids gpurun_out/r03af_fixed32_ab.txt
echo R03AF_OK
