#!/bin/bash
# Round profile: bench lines for configs 2/3/5, rocprofv3 kernel stats of the same
# commands, and FETCH_SIZE / WRITE_SIZE PMC passes (separate runs, kernel-trace only).
# Usage: OUT=gpurun_out/prof_rNN TAG=rNN bash tools/profile_round.sh
set -o pipefail
OUT=${OUT:-gpurun_out/prof}
R=$(pwd)
mkdir -p "$OUT"
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"; local rc=$?
  [ $rc -eq 0 ] || { echo "STEP $name failed rc=$rc"; tail -5 "$OUT/$name.err"; exit 1; }
}
prof() {  # name, args for bench.py
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$R/$OUT/$name" -o run -- python3 "$R/bench.py" "$@" > "$R/$OUT/$name.log" 2>&1) || { echo "PROF $name failed"; tail -5 "$R/$OUT/$name.log"; exit 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv \
       -d "$R/$OUT/${name}_$c" -o pmc -- python3 "$R/bench.py" "$@" > "$R/$OUT/${name}_$c.log" 2>&1) || { echo "PMC $name $c failed"; tail -5 "$R/$OUT/${name}_$c.log"; exit 1; }
  done
}
run bench_fixed32 400 python3 bench.py
cat "$OUT/bench_fixed32.out"
run bench_csr 400 python3 bench.py --config csr --steps 10 --warmup 3 --no-cpu-baseline
cat "$OUT/bench_csr.out"
run bench_fixed4096 400 python3 bench.py --config fixed4096 --steps 10 --warmup 3 --no-cpu-baseline
cat "$OUT/bench_fixed4096.out"
prof fixed32 --steps 10 --warmup 3 --no-cpu-baseline
prof csr --config csr --steps 5 --warmup 2 --no-cpu-baseline
prof fixed4096 --config fixed4096 --steps 5 --warmup 2 --no-cpu-baseline
echo PROFILE_ROUND_OK
