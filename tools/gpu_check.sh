#!/bin/bash
# One GPU round-trip: smoke, GPU parity tests, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out/check}
mkdir -p "$OUT"
R=$(pwd)
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && echo SMOKE_OK &&
timeout -k 10 900 python3 -m pytest tests -x -q -m gpu ${PYTEST_ARGS} > "$OUT/pytest_gpu.log" 2>&1 ; rc=$?; tail -5 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] &&
timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && cat "$OUT/bench.json" &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$OUT/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$R/$OUT/prof.log" 2>&1) && echo PROF_OK
