#!/bin/bash
# round 3 (session 2): persistent half-line line-DMA kernel at 16 waves/CU (4 per SIMD, 4
# tiles per wave, no drain) against the product (config 5), digest-checked first
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/lab_ab.py lines --variants 0:0 3:16 1:8 3:8 --reps 7 > gpurun_out/r03ae_lines_ab.json 2> gpurun_out/r03ae_lines_ab.err
python3 -c "
import json; d=json.load(open('gpurun_out/r03ae_lines_ab.json'))
for v,r in d['results'].items(): print(v, r['verify'], round(r['median_us'],1), round(r['min_us'],1))"
echo R03AE_OK
