#!/bin/bash
# Round 3 (session 2): import profile and the per-config issue / wait PMC breakdown.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 bash tools/gpu/r03_import_prof.sh || exit 1
OUT=gpurun_out/pmc_r03ab bash tools/pmc_round.sh fixed32 csr fixed4096 ralledata || exit 1
echo R03AB_OK
