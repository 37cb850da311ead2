#!/bin/bash
set -o pipefail
OUT=${OUT:-gpurun_out/r3}
mkdir -p "$OUT"
timeout -k 10 900 python3 -m pytest tests -x -q -m gpu > "$OUT/pytest_gpu.log" 2>&1; rc=$?; tail -15 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] &&
timeout -k 10 300 python3 tools/variants.py --config csr --variants 0,10,3 --rounds 3 --reps 5 > "$OUT/csr.log" 2>&1; cat "$OUT/csr.log" &&
timeout -k 10 300 python3 tools/variants.py --config fixed4096 --variants 0,10 --rounds 3 --reps 5 > "$OUT/fixed4096.log" 2>&1; cat "$OUT/fixed4096.log" &&
timeout -k 10 300 python3 tools/variants.py --config fixed32 --variants 0,4 --rounds 7 --reps 10 > "$OUT/fixed32.log" 2>&1; cat "$OUT/fixed32.log"
