#!/bin/bash
# round 3 (session 2): fixed32 headline with THREE keys per lane in one asm statement
# (key k hashed after its own loads) -- parity tests, then A/B against HEAD (two keys)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03al_pytest_parity.txt 2>&1
tail -2 gpurun_out/r03al_pytest_parity.txt
timeout -k 10 300 python -u tools/ab_libs.py --config fixed32 --libs k2hash_amd/lib/ab/HEAD/libk2hash_amd.so --rounds 15 --reps 20 > gpurun_out/r03al_fixed32_ab.txt 2>&1
timeout -k 10 300 python -u tools/ab_libs.py --config fixed32 --libs k2hash_amd/lib/ab/HEAD/libk2hash_amd.so --rounds 15 --reps 20 >> gpurun_out/r03al_fixed32_ab.txt 2>&1
grep -v amdgpu.ids gpurun_out/r03al_fixed32_ab.txt
echo R03AL_OK
