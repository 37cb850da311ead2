#!/bin/bash
# Issue / wait breakdown of each bench config's dominant kernel (round 3+): two PMC passes
# per config (one counter group per run, --kernel-trace only beside --pmc), summarised by
# tools/pmc_table.py into VALU utilisation, waves per SIMD and the wait fraction.
#   OUT=gpurun_out/pmc_rNN bash tools/pmc_round.sh [config ...]
set -o pipefail
OUT=${OUT:-gpurun_out/pmc_round}
R=$(pwd)
mkdir -p "$OUT"
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL"
P2="SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM"
for c in ${*:-fixed32 csr fixed4096 ralledata}; do
  case $c in
    fixed32) args="--no-secondary --no-cpu-baseline"; rx="fnv_" ;;
    ralledata) args="--config ralledata --no-cpu-baseline"; rx="ralledata" ;;
    *) args="--config $c --no-cpu-baseline"; rx="fnv_" ;;
  esac
  for p in 1 2; do
    eval "ctr=\$P$p"
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr --kernel-include-regex "$rx" \
       --output-format csv -d "$R/$OUT/$c/${c}_p$p" -o pmc -- python3 "$R/bench.py" $args \
       --steps 10 --warmup 2 --no-verify > "$R/$OUT/${c}_p$p.log" 2>&1) || { echo "PMC $c p$p failed"; tail -5 "$R/$OUT/${c}_p$p.log"; exit 1; }
  done
  python3 "$R/tools/pmc_table.py" "$R/$OUT/$c" "$rx" > "$R/$OUT/${c}_table.txt" || exit 1
  cat "$R/$OUT/${c}_table.txt"
done
echo PMC_ROUND_OK
