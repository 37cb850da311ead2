#!/bin/bash
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_archive.py tests/test_import.py -m gpu -x -q --timeout 300 --timeout-method thread -k "host or prehash" > gpurun_out/r02c_pytest.txt 2>&1
tail -3 gpurun_out/r02c_pytest.txt
timeout -k 10 400 python -u bench.py > gpurun_out/r02c_bench.json 2> gpurun_out/r02c_bench.err
python -c "import json;d=json.load(open('gpurun_out/r02c_bench.json'));print(json.dumps(d['secondary']['host'],indent=1)); print(d['roofline']['frac'])"
