#!/bin/bash
# quick: GPU parity subset (-k filter) + variant timings given as "config:variants" pairs
set -o pipefail
OUT=${OUT:-gpurun_out/q}
mkdir -p "$OUT"
timeout -k 10 900 python3 -m pytest tests -x -q -m gpu ${K:+-k "$K"} > "$OUT/pytest_gpu.log" 2>&1; rc=$?; tail -4 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit 1
for cv in $RUNS; do
  c=${cv%%:*}; v=${cv#*:}
  timeout -k 10 300 python3 tools/variants.py --config $c --variants $v --rounds ${ROUNDS:-3} --reps ${REPS:-5} > "$OUT/$c.log" 2>&1; rc=$?; grep -v amdgpu.ids "$OUT/$c.log"; [ $rc -eq 0 ] || exit 1
done
