#!/bin/bash
# The driver's own bench command (python bench.py, defaults) under rocprofv3 kernel and
# marker traces.  bench.py (K2H_BENCH_MARKERS=1) wraps the synchronised timed region of the
# headline and of every secondary in a roctx range "timed:<label>", so every figure in the
# line is recomputed from the kernels inside its own range, in the same process
# (tools/summarize_line_profile.py).  No counters here (--pmc runs are
# tools/profile_round.sh's, one group per run).
#   OUT=gpurun_out/line_rNN bash tools/profile_line.sh [extra bench.py args]
set -o pipefail
OUT=${OUT:-gpurun_out/line}
R=$(pwd)
mkdir -p "$OUT"
export K2H_BENCH_MARKERS=1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --marker-trace --stats \
   --output-format csv -d "$R/$OUT/trace" -o run -- python3 "$R/bench.py" "$@" > "$R/$OUT/bench.log" 2>&1) \
   || { echo "LINE PROFILE failed"; tail -20 "$R/$OUT/bench.log"; exit 1; }
grep '^{' "$R/$OUT/bench.log" > "$R/$OUT/bench_line.json" || { echo "no bench line"; exit 1; }
echo LINE_PROFILE_OK
