#!/bin/bash
# Round 3: the whole GPU suite, the default bench line, and the round profile of every
# bench config (rocprofv3 timed window + PMC traffic / VALU passes).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r03m_pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/r03m_pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/r03m_pytest_gpu.txt
timeout -k 10 400 python bench.py > gpurun_out/r03m_bench.json 2> gpurun_out/r03m_bench.err || { tail -20 gpurun_out/r03m_bench.err; exit 1; }
OUT=gpurun_out/prof_r03m bash tools/profile_round.sh fixed32 csr fixed4096 fixed32_1g ralledata fixed32_index || exit 1
timeout -k 10 600 bash tools/gpu/r03_import_prof.sh || exit 1
echo R03M_OK
