#!/bin/bash
# import_probe_times.sh for the mdbm form (tools/import_step.py --mdbm; the tree verifies
# first, probe libraries are timed only).
#   gpurun -- 'OUT=r06ab LIBS=k2hash_amd/lib/probe/a.so bash tools/gpu/import_probe_times_mdbm.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/${OUT:-import_probe_mdbm}
mkdir -p $O
for L in tree ${LIBS//,/ }; do
  n=$(basename $L .so); A=""; [ "$L" != tree ] && A="--lib $R/$L"
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$n -o run -- python3 $R/tools/import_step.py --mdbm --rounds 3 $A ${A:+--no-parity} > $O/$n.log 2>&1) || { tail $O/$n.log; exit 1; }
  echo "== $n: $(grep -h mdbm_ms $O/$n.log | cut -c1-80)"
  python3 tools/kernel_trace_table.py $O/$n/run_kernel_trace.csv "tsv_" 10 | cut -c1-100
done
echo IMPORT_PROBE_TIMES_OK
