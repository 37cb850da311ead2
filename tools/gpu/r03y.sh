#!/bin/bash
# round 3 (session 2): lean line-DMA kernel (product candidate) -- GPU suite, then A/B
# against the HEAD build on config 5 (h1, and h1+h2)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03y_pytest_gpu.txt 2>&1
tail -2 gpurun_out/r03y_pytest_gpu.txt
timeout -k 10 300 python -u tools/ab_libs.py --config fixed4096 --libs k2hash_amd/lib/ab/HEAD/libk2hash_amd.so --rounds 9 --reps 10 > gpurun_out/r03y_lines_ab.txt 2>&1
timeout -k 10 300 python -u tools/ab_libs.py --config fixed4096 --second --libs k2hash_amd/lib/ab/HEAD/libk2hash_amd.so --rounds 7 --reps 10 >> gpurun_out/r03y_lines_ab.txt 2>&1
grep -v amdgpu.ids gpurun_out/r03y_lines_ab.txt
echo R03Y_OK
