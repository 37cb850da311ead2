#!/bin/bash
# PMC of the TSV device-scan kernels (instruction mix, wave cycles)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/imp_pmc
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM --kernel-include-regex "tsv_" --output-format csv -d gpurun_out/imp_pmc -o run -- python3 -u tools/import_rate.py --reps 1 > gpurun_out/imp_pmc/rate.json 2> gpurun_out/imp_pmc/err.txt
find gpurun_out/imp_pmc -name "*counter_collection.csv" | head -1
