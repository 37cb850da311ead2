#!/bin/bash
# k2himport profile: kernel trace + stats, then FETCH_SIZE / WRITE_SIZE / SQ passes (one group per run)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# MDBM=1: the same over the mdbm form of the workload (tools/import_step.py --mdbm) into prof_import_mdbm
R=$(pwd); O=$R/gpurun_out/prof_import${MDBM:+_mdbm}
A="${MDBM:+--mdbm --rounds 3}"
rm -rf $O; mkdir -p $O
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/import_step.py --calls 10 $A > $O/trace.log 2>&1)
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "tsv_|rocprim" --output-format csv -d $O/pmc$i -o pmc -- python3 $R/tools/import_step.py --calls 4 $A > $O/pmc$i.log 2>&1)
done
echo IMPORT_PROFILE_OK
