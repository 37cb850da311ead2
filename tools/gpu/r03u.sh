#!/bin/bash
# round 3: CSR setup lab A/B on the new product (offsets batched): 9 (seed table computed,
# not loaded), 10 (9 + each wave's span DMA before the block barrier)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/lab_ab.py csr --variants 0 9 10 --reps 7 > gpurun_out/r03u_csr_ab.json 2> gpurun_out/r03u_csr_ab.err || { tail -20 gpurun_out/r03u_csr_ab.err; exit 1; }
cat gpurun_out/r03u_csr_ab.json
echo R03U_OK
