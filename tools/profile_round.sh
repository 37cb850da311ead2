#!/bin/bash
# Round profile: rocprofv3 kernel trace + stats of the bench command for each config
# (timed window = the last --steps dispatches of the dominant kernel), then PMC passes
# (one counter group per run, --kernel-trace only beside --pmc): FETCH_SIZE, WRITE_SIZE,
# and the SQ instruction counters.
# Usage: OUT=gpurun_out/prof_rNN bash tools/profile_round.sh [config ...]
set -o pipefail
OUT=${OUT:-gpurun_out/prof}
R=$(pwd)
mkdir -p "$OUT"
CONFIGS=${*:-fixed32 csr fixed4096 fixed32_1g}
prof() {  # name, args for bench.py
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$R/$OUT/$name" -o run -- python3 "$R/bench.py" "$@" > "$R/$OUT/$name.log" 2>&1) || { echo "PROF $name failed"; tail -5 "$R/$OUT/$name.log"; exit 1; }
  grep '^{' "$R/$OUT/$name.log" > "$R/$OUT/bench_$name.out" || true
  local short="--steps 10 --warmup 2 --no-verify"  # warmed (150 ms): the clock of the timed region
  local i=0
  for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES"; do
    i=$((i+1))
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "fnv_|ralledata" \
       --output-format csv -d "$R/$OUT/${name}_pmc$i" -o pmc -- python3 "$R/bench.py" "$@" $short > "$R/$OUT/${name}_pmc$i.log" 2>&1) \
       || { echo "PMC $name pass $i ($c) failed"; tail -5 "$R/$OUT/${name}_pmc$i.log"; exit 1; }
  done
}
for cfg in $CONFIGS; do
  case $cfg in
    fixed32) prof fixed32 --no-secondary --no-cpu-baseline ;;
    fixed32_index) prof fixed32_index --index --no-secondary --no-cpu-baseline ;;
    *) prof "$cfg" --config "$cfg" --steps 20 --warmup 3 --no-cpu-baseline ;;
  esac
  echo "profiled $cfg"
done
echo PROFILE_ROUND_OK
