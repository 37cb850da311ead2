#!/bin/bash
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 76 89; do
timeout -k 10 100 python -u tools/ralle_phases.py --variant $v > gpurun_out/ph$v.json
python3 -c "
import json; d=json.load(open('gpurun_out/ph$v.json'))
print($v, round(d['kernel_ms'],3), {k:round(d[k]['mean_us'],2) for k in d if isinstance(d[k],dict)}, round(d['resident_blocks_mean']))"
done
timeout -k 10 300 python -u tools/ralle_ab.py --variants 73,0,88,0,88,0,88
