#!/bin/bash
# kernel times of the TSV device scan (rocprofv3 stats over tools/import_rate.py)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/imp_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/imp_prof -o run -- python3 -u tools/import_rate.py --reps 3 > gpurun_out/imp_prof/rate.json
find gpurun_out/imp_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cut -c1-200 {} | head -14
