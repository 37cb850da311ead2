#!/bin/bash
# Per-kernel times of the k2himport kernels for each probe library in LIBS (timing only:
# probes may compute wrong results by design), and the tree's, under rocprofv3 --kernel-trace.
#   gpurun -- 'OUT=r06z LIBS=k2hash_amd/lib/probe/a.so,... bash tools/gpu/import_probe_times.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/${OUT:-import_probe}
mkdir -p $O
for L in tree ${LIBS//,/ }; do
  n=$(basename $L .so); A=""; [ "$L" != tree ] && A="--lib $R/$L"
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$n -o run -- python3 $R/tools/import_step.py --calls 10 $A > $O/$n.log 2>&1) || { tail $O/$n.log; exit 1; }
  echo "== $n: $(tail -1 $O/$n.log)"
  python3 tools/kernel_trace_table.py $O/$n/run_kernel_trace.csv "tsv_" 10 | cut -c1-100
done
echo IMPORT_PROBE_TIMES_OK
