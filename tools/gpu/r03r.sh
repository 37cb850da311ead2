#!/bin/bash
# round 3: CSR setup-latency lab A/B: 2 (offset loads together), 3 (wave 0 offsets while
# waves 1-3 DMA), 4 (3 + wave 0 sorts alone)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/lab_ab.py csr --variants 0 2 3 4 --reps 7 > gpurun_out/r03r_csr_ab.json 2> gpurun_out/r03r_csr_ab.err || { tail -20 gpurun_out/r03r_csr_ab.err; exit 1; }
cat gpurun_out/r03r_csr_ab.json
echo R03R_OK
