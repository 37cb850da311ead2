#!/bin/bash
# host-side API times of the TSV device scan (rocprofv3 --hip-trace --stats)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/imp_api
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats -d gpurun_out/imp_api -o run -- python3 -u tools/import_rate.py --reps 3 > gpurun_out/imp_api/rate.json 2> gpurun_out/imp_api/err.txt
