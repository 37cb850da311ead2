#!/bin/bash
# Round 4: per-kernel import times, tree vs HEAD library
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/r04f
mkdir -p $O
for lib in tree head; do
  arg=""; [ $lib = head ] && arg=$R/k2hash_amd/lib/probe/head.so
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$lib -o run -- python3 $R/tools/import_probe.py $arg > $O/$lib.log 2>&1) || { tail $O/$lib.log; exit 1; }
  echo "== $lib"; python3 tools/kernel_trace_table.py $O/$lib/run_kernel_trace.csv "tsv_" 10
done
echo R04F_OK
