#!/bin/bash
# Round 3: single-read TSV import scan (per-call time, rocprof trace + PMC); CSR
# register-staged lab A/B after the store-base fix.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 bash tools/gpu/r03_import_prof.sh || exit 1
timeout -k 10 240 python tools/lab_ab.py csr --variants 0 1 --reps 7 > gpurun_out/r03d_csr_ab.json 2> gpurun_out/r03d_csr_ab.err || { tail -20 gpurun_out/r03d_csr_ab.err; exit 1; }
cat gpurun_out/r03d_csr_ab.json
echo R03D_OK
