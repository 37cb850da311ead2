#!/bin/bash
# PMC comparison of lab variants: one rocprofv3 --pmc run per (variant, counter group).
# usage: OUT=gpurun_out/pmcv CONFIG=csr bash tools/pmc_variants.sh 0 64 61
set -o pipefail
OUT=${OUT:-gpurun_out/pmcv}
CONFIG=${CONFIG:-csr}
KREGEX=${KREGEX:-fnv_}
R=$(pwd)
mkdir -p "$OUT"
GROUPS_=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAVES")
for v in "$@"; do
  i=0
  for g in "${GROUPS_[@]}"; do
    i=$((i+1))
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $g --kernel-include-regex "$KREGEX" \
       --output-format csv -d "$R/$OUT/v${v}_g$i" -o pmc -- python3 "$R/tools/run_variant.py" --config $CONFIG --variant $v \
       > "$R/$OUT/v${v}_g$i.log" 2>&1) || { echo "PMC v$v g$i failed"; tail -5 "$R/$OUT/v${v}_g$i.log"; exit 1; }
  done
  echo "pmc variant $v ok"
done
