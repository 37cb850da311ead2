#!/bin/bash
# RALLEDATA gather form: parity tests, A/B against the group kernel, kernel stats
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ralledata.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r02f_pytest.txt 2>&1 || { tail -30 gpurun_out/r02f_pytest.txt; exit 1; }
tail -3 gpurun_out/r02f_pytest.txt
timeout -k 10 300 python -u tools/ralle_ab.py --variants 73,0 > gpurun_out/r02f_ab.txt 2>&1 || { tail -20 gpurun_out/r02f_ab.txt; exit 1; }
cat gpurun_out/r02f_ab.txt
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r02f_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config ralledata --steps 20 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r02f_bench.log 2>&1)
grep '^{' gpurun_out/r02f_bench.log | tail -1 | cut -c1-400
