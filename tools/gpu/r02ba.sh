#!/bin/bash
# Round-2 session y: GPU suite on the tree with lean2's setup-phase priority and single-wave
# class scan, then the CSR round profile (timed window + PMC traffic / VALU).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02ba_pytest_gpu.txt 2>&1 || { tail -5 gpurun_out/r02y2_pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/r02ba_pytest_gpu.txt
OUT=gpurun_out/prof_r02ba bash tools/profile_round.sh csr
