#!/bin/bash
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/copy_floor | tee gpurun_out/r02j_copy_floor.txt
timeout -k 10 120 ./tools/copy_floor 1800000000 1800000000 | tee -a gpurun_out/r02j_copy_floor.txt
timeout -k 10 200 python -u tools/ralle_ab.py --variants 74,0
