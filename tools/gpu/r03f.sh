#!/bin/bash
# Round 3: wall time per TSV import call (three runs) and its HIP API breakdown.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do timeout -k 10 120 python tools/import_step.py --calls 50 || exit 1; done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --runtime-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03f_rt -o rt -- python3 $GRAFT_REPO_ROOT/tools/import_step.py --calls 20 > $GRAFT_REPO_ROOT/gpurun_out/r03f_rt.log 2>&1) || exit 1
echo R03F_OK
