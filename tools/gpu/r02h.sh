#!/bin/bash
# RALLEDATA gather form v2: parity tests, A/B against the group kernel, PMC
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ralledata.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r02h_pytest.txt 2>&1 || { tail -30 gpurun_out/r02h_pytest.txt; exit 1; }
tail -2 gpurun_out/r02h_pytest.txt
timeout -k 10 300 python -u tools/ralle_ab.py --variants 73,74,0 > gpurun_out/r02h_ab.txt 2>&1 || { tail -20 gpurun_out/r02h_ab.txt; exit 1; }
cat gpurun_out/r02h_ab.txt
OUT=gpurun_out/pmc_ralle3 CONFIG=ralledata KREGEX=ralledata bash tools/pmc_variants.sh 0
python3 tools/pmc_table.py gpurun_out/pmc_ralle3 ralledata
