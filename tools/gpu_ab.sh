#!/bin/bash
# GPU parity (full -m gpu suite unless K is set) + in-process A/B of the tree's library
# against the libraries named in LIBS, for each config in CONFIGS.
set -o pipefail
OUT=${OUT:-gpurun_out/ab}
mkdir -p "$OUT"
timeout -k 10 900 python3 -m pytest tests -x -q -m gpu ${K:+-k "$K"} > "$OUT/pytest_gpu.log" 2>&1; rc=$?; tail -4 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit 1
for c in ${CONFIGS:-csr fixed32 fixed4096}; do
  timeout -k 10 300 python3 tools/ab_libs.py --config $c --libs "$LIBS" --rounds ${ROUNDS:-5} --reps ${REPS:-10} ${ABARGS} > "$OUT/$c.log" 2>&1; rc=$?; grep -v amdgpu.ids "$OUT/$c.log"; [ $rc -eq 0 ] || exit 1
done
