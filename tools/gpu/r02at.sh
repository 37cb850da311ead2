#!/bin/bash
# RALLEDATA gather kernel: LDS alignment / conflict counters (one SQ group)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/ralle_lds; rm -rf $O; mkdir -p $O
(cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --kernel-include-regex "ralledata" --output-format csv -d $O -o pmc -- python3 $R/tools/run_variant.py --config ralledata --variant 0 > $O/log.txt 2>&1)
echo RALLE_LDS_OK
