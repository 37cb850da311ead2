#!/bin/bash
# Round 4: mdbm on the TSV machinery -- import GPU tests, then TSV timing vs HEAD
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_import.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04e_pytest_import.txt 2>&1 || { tail -40 gpurun_out/r04e_pytest_import.txt; exit 1; }
tail -2 gpurun_out/r04e_pytest_import.txt
timeout -k 10 300 python3 tools/import_step.py --ab k2hash_amd/lib/probe/head.so --rounds 7 --calls 10 2>&1 | grep -v Warn
echo R04E_OK
