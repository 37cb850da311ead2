#!/bin/bash
# PMC passes on the CSR and 4 KiB bench configs: VALU / LDS stall / clock counters.
set -o pipefail
OUT=${OUT:-gpurun_out/pmc_csr}
mkdir -p "$OUT"
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL"
P2="SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM"
for cfg in "${CFGS[@]:-csr:0 csr:19 fixed4096:0}"; do :; done
for cv in ${CFGS:-csr:0 csr:19 fixed4096:0}; do
  c=${cv%%:*}; v=${cv##*:}
  for p in 1 2; do
    eval "ctr=\$P$p"
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $ctr --kernel-include-regex fnv_ \
       --output-format csv -d "$OLDPWD/$OUT/${c}_v${v}_p$p" -o pmc -- python3 "$OLDPWD/bench.py" --config $c --variant $v \
       --steps 3 --warmup 2 --warm-ms 0 --no-cpu-baseline > "$OLDPWD/$OUT/${c}_v${v}_p$p.log" 2>&1) || { echo "PMC $c v$v p$p failed"; tail -5 "$OUT/${c}_v${v}_p$p.log"; exit 1; }
  done
done
echo PMC_CSR_OK
