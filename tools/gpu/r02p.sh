#!/bin/bash
# RALLEDATA profile (trace + PMC) of the final gather kernel
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/prof_r02p bash tools/profile_round.sh ralledata
grep '^{' gpurun_out/prof_r02p/ralledata.log | tail -1 | cut -c1-300
