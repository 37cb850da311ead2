#!/bin/bash
# Issue / wait breakdown (VALU, SALU, LDS instructions, waves, wave cycles, SQ_WAIT_ANY) of
# the bench kernels of every config, one rocprofv3 --pmc pass per config (kernel trace only
# beside it), tabulated by tools/kernel_pmc_table.py.
#   gpurun -- 'OUT=r05ao bash tools/gpu/issue_wait.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/${OUT:-issue_wait}
mkdir -p $O
for cfg in fixed32 csr fixed4096 ralledata; do
  args="--config $cfg --steps 10 --warmup 2 --no-verify --no-cpu-baseline --no-secondary"
  (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES \
     --kernel-include-regex "fnv_|ralledata" --output-format csv -d $O/$cfg -o pmc -- python3 $R/bench.py $args > $O/$cfg.log 2>&1) \
     || { echo "PMC $cfg failed"; tail -5 $O/$cfg.log; exit 1; }
  echo "== $cfg"
  python3 tools/kernel_pmc_table.py "fnv_|ralledata" $O/$cfg 2>&1 | cut -c1-150
done
echo ISSUE_WAIT_OK
