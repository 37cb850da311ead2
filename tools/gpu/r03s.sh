#!/bin/bash
# round 3: CSR setup-latency lab A/B: 2 (offset loads together), 6 (asm offset loads,
# scalar seed table), 7 (6 + DMA before the offset wait), 8 (offsets + tile bounds in one latency)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/lab_ab.py csr --variants 0 2 6 7 8 --reps 7 > gpurun_out/r03s_csr_ab.json 2> gpurun_out/r03s_csr_ab.err || { tail -20 gpurun_out/r03s_csr_ab.err; exit 1; }
cat gpurun_out/r03s_csr_ab.json
echo R03S_OK
