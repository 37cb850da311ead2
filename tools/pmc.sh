#!/bin/bash
# PMC passes (one counter group per pass, --kernel-trace only beside --pmc) for a
# python command, e.g.  OUT=gpurun_out/pmc tools/pmc.sh bench.py --steps 5 --warmup 2 --no-cpu-baseline
# Writes CSVs under $OUT/<pass>/.  Each pass has its own time limit; stops at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out/pmc}
R=$(pwd)
KREGEX=${KREGEX:-fnv_}
mkdir -p "$OUT"
if [ -n "$PMC_PASSES" ]; then IFS=';' read -r -a PASSES <<< "$PMC_PASSES"; else PASSES=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU"
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
); fi
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc $p --kernel-include-regex "$KREGEX" \
     --output-format csv -d "$R/$OUT/pass$i" -o pmc -- python3 "$R/$@" > "$R/$OUT/pass$i.log" 2>&1) || { echo "PMC pass $i ($p) failed"; tail -5 "$R/$OUT/pass$i.log"; exit 1; }
done
echo PMC_OK
