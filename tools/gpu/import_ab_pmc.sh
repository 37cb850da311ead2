#!/bin/bash
# import_ab.sh, then the PMC passes (FETCH_SIZE, WRITE_SIZE, VALU/SALU) for every library in
# LIBS too, not only the tree's, so that a traffic A/B compares like with like.
#   gpurun -- 'OUT=r06u LIBS=k2hash_amd/lib/probe/a.so,k2hash_amd/lib/probe/b.so bash tools/gpu/import_ab_pmc.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/${OUT:-import_ab}
bash tools/gpu/import_ab.sh || exit 1
for L in ${LIBS//,/ }; do
  n=$(basename $L .so); i=0
  for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES"; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "tsv_" --output-format csv -d $O/${n}_pmc$i -o pmc -- python3 $R/tools/import_step.py --lib $R/$L --calls 4 > $O/${n}_pmc$i.log 2>&1) || { tail $O/${n}_pmc$i.log; exit 1; }
  done
  echo "== $n"
  python3 tools/kernel_pmc_table.py "tsv_" $O/${n}_pmc1 $O/${n}_pmc2 $O/${n}_pmc3 2>&1 | cut -c1-140
done
echo IMPORT_AB_PMC_OK
