#!/bin/bash
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ralledata.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02n_pytest.txt 2>&1 || { tail -30 gpurun_out/r02n_pytest.txt; exit 1; }
tail -1 gpurun_out/r02n_pytest.txt
timeout -k 10 100 python -u tools/ralle_phases.py --variant 76 > gpurun_out/ph76b.json
python3 -c "
import json; d=json.load(open('gpurun_out/ph76b.json'))
print(round(d['kernel_ms'],3), {k:round(d[k]['mean_us'],2) for k in d if isinstance(d[k],dict)}, round(d['resident_blocks_mean']))"
timeout -k 10 300 python -u tools/ralle_ab.py --variants 73,0,81,0
