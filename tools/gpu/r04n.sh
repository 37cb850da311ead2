#!/bin/bash
# Round 4: import pass A/B issue and wait counters, tree vs HEAD (probe/prev.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/r04n
mkdir -p $O
P=k2hash_amd/lib/probe
for lib in tree prev; do
  arg=""; [ $lib != tree ] && arg="--lib $R/$P/$lib.so"
  i=0
  for c in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS" "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM"; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "tsv_" --output-format csv -d $O/$lib$i -o pmc -- python3 $R/tools/import_step.py --calls 4 $arg > $O/$lib$i.log 2>&1) || { tail $O/$lib$i.log; exit 1; }
  done
  echo "== $lib"
  python3 tools/kernel_pmc_table.py "tsv_" $O/${lib}1 $O/${lib}2 2>&1 | cut -c1-140
done
echo R04N_OK
