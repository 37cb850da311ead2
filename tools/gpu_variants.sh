#!/bin/bash
set -o pipefail
OUT=${OUT:-gpurun_out/var}
mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1
timeout -k 10 600 python3 tools/variants.py --config fixed32 --variants 4,5,6,1 --rounds 5 --reps 10 > "$OUT/fixed32.log" 2>&1; cat "$OUT/fixed32.log" &&
timeout -k 10 600 python3 tools/variants.py --config csr --variants 0 --rounds 3 --reps 5 > "$OUT/csr.log" 2>&1; cat "$OUT/csr.log" &&
timeout -k 10 600 python3 tools/variants.py --config fixed4096 --variants 0 --rounds 3 --reps 5 > "$OUT/fixed4096.log" 2>&1; cat "$OUT/fixed4096.log" &&
timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; cat "$OUT/bench.json" &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/$OUT/prof" -o run -- python3 "$OLDPWD/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$OLDPWD/$OUT/prof.log" 2>&1) && echo PROF_OK &&
OUT=$OUT/pmc bash tools/pmc.sh bench.py --steps 5 --warmup 2 --no-cpu-baseline
