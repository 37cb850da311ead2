#!/bin/bash
# Round-2 final tree: round profile of every bench config (rocprofv3 timed window + PMC
# traffic / VALU passes), then the default bench line.
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/prof_r02bd bash tools/profile_round.sh fixed32 csr fixed4096 fixed32_1g ralledata fixed32_index || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r02bd_bench.json 2> gpurun_out/r02bd_bench.err || exit 1
echo R02BD_OK
