#!/bin/bash
# import GPU tests (incl. the bench workload digest), then the default bench line
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_import.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/imp_tests.txt 2>&1
tail -3 gpurun_out/imp_tests.txt
timeout -k 10 400 python -u bench.py > gpurun_out/r02aq_bench.json 2> gpurun_out/r02aq_bench.err
python3 -c "
import json; d=json.load(open('gpurun_out/r02aq_bench.json'))
print(d['value'], d['roofline']['frac'])
i=d['secondary']['import']; print(json.dumps(i)[:600])"
