#!/bin/bash
# Round 4: import probe -- tsv_b with vs without the fused prehash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/r04c
mkdir -p $O
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/tools/import_probe.py > $O/trace.log 2>&1) || { tail $O/trace.log; exit 1; }
python3 tools/kernel_trace_table.py $O/trace/run_kernel_trace.csv "tsv_" 10
echo R04C_OK
