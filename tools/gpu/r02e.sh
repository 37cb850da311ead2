#!/bin/bash
# clock probe (s_memtime per wave) + RALLEDATA profile with its own kernel in the PMC regex
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/clock_probe.py --json gpurun_out/clock_probe.json
OUT=gpurun_out/prof_r02e bash tools/profile_round.sh ralledata
