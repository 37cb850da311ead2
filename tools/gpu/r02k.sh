#!/bin/bash
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ralledata.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02k_pytest.txt 2>&1 || { tail -30 gpurun_out/r02k_pytest.txt; exit 1; }
tail -1 gpurun_out/r02k_pytest.txt
timeout -k 10 300 python -u tools/ralle_ab.py --variants 73,0
