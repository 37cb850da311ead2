#!/bin/bash
# full GPU suite + smoke on the current tree
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r02as_pytest_gpu.txt 2>&1
tail -3 gpurun_out/r02as_pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()"
