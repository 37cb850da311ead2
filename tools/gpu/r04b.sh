#!/bin/bash
# Round 4: per-kernel issue/wait breakdown of the k2himport TSV device scan (import_step.py, 8M records)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/r04b
mkdir -p $O
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM"
P2="SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM"
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/import_step.py --calls 10 > $O/trace.log 2>&1) || { tail $O/trace.log; exit 1; }
for p in 1 2; do
  eval "ctr=\$P$p"
  (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr --kernel-include-regex "tsv_" --output-format csv -d $O/p$p -o pmc -- python3 $R/tools/import_step.py --calls 4 > $O/p$p.log 2>&1) || { echo "pass $p failed"; tail $O/p$p.log; exit 1; }
done
python3 tools/kernel_pmc_table.py tsv_ $O/p1 $O/p2 | tee $O/table.txt
grep tsv_ $O/trace/run_kernel_stats.csv | cut -c1-200
echo R04B_OK
