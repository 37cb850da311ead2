#!/bin/bash
# PMC counters of the RALLEDATA gather (0) and group (73) assembly kernels
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ralle CONFIG=ralledata KREGEX=ralledata bash tools/pmc_variants.sh 0 73
python3 tools/pmc_table.py gpurun_out/pmc_ralle ralledata
