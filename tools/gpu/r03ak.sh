#!/bin/bash
# round 3 (session 2): CSR pair walk with unchecked runs before the wave's first switch and
# between its last switch and first end -- GPU suite, then A/B against HEAD on config 3
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ak_pytest_gpu.txt 2>&1
tail -2 gpurun_out/r03ak_pytest_gpu.txt
timeout -k 10 400 python -u tools/ab_libs.py --config csr --libs k2hash_amd/lib/ab/HEAD/libk2hash_amd.so --rounds 9 --reps 5 > gpurun_out/r03ak_csr_ab.txt 2>&1
timeout -k 10 400 python -u tools/ab_libs.py --config csr --second --libs k2hash_amd/lib/ab/HEAD/libk2hash_amd.so --rounds 5 --reps 5 >> gpurun_out/r03ak_csr_ab.txt 2>&1
grep -v amdgpu.ids gpurun_out/r03ak_csr_ab.txt
echo R03AK_OK
