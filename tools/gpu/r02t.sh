#!/bin/bash
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmc_4k CONFIG=fixed4096 bash tools/pmc_variants.sh 0
python3 tools/pmc_table.py gpurun_out/pmc_4k
OUT=gpurun_out/pmc_f32 CONFIG=fixed32 bash tools/pmc_variants.sh 0
python3 tools/pmc_table.py gpurun_out/pmc_f32
