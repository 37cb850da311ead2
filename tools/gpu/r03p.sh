#!/bin/bash
# round 3: RALLEDATA lab A/B, variants 3, 4 (next window only for crossing pieces; table entry one piece ahead)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python tools/lab_ab.py ralle --variants 0 3 4 --reps 9 > gpurun_out/r03p_ralle_ab.json 2> gpurun_out/r03p_ralle_ab.err || { tail -20 gpurun_out/r03p_ralle_ab.err; exit 1; }
cat gpurun_out/r03p_ralle_ab.json
echo R03P_OK
