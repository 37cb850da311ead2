#!/bin/bash
# Round-end evidence: the GPU suite, the default bench line, the round profile of every bench
# config (rocprofv3 timed window + PMC traffic / VALU passes) and the k2himport profile.
#   gpurun -- 'TAG=r04zb bash tools/gpu/final.sh'   (then tools/summarize_profiles.py and
#   tools/summarize_import_profile.py on gpurun_out/prof_<TAG> and gpurun_out/prof_import)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-final}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/${T}_pytest_gpu.txt
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
OUT=gpurun_out/prof_${T} bash tools/profile_round.sh fixed32 csr fixed4096 fixed32_1g ralledata fixed32_index || exit 1
timeout -k 10 600 bash tools/gpu/import_prof.sh || exit 1
echo ${T}_OK
