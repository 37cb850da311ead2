#!/bin/bash
# Round 3: CSR register-staged lab kernel A/B after the store-base fix.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python tools/lab_ab.py csr --variants 0 1 --reps 7 > gpurun_out/r03c_csr_ab.json 2> gpurun_out/r03c_csr_ab.err || { tail -20 gpurun_out/r03c_csr_ab.err; exit 1; }
cat gpurun_out/r03c_csr_ab.json
echo R03C_OK
