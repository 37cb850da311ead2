#!/bin/bash
# Round-end evidence, in two gpurun calls (each well under the 20-minute limit):
#   PART=1: the GPU suite, the default bench line, the line profile (the driver's command
#           under rocprofv3 with a roctx range per entry, tools/profile_line.sh) and the
#           k2himport profile;
#   PART=2: the round profile of every bench config (timed window + PMC traffic / VALU).
#   gpurun -- 'TAG=r06final PART=1 bash tools/gpu/final.sh'   (then tools/summarize_line_profile.py,
#   tools/summarize_profiles.py and tools/summarize_import_profile.py on gpurun_out/)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-final}
if [ "${PART:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest_gpu.txt; exit 1; }
  tail -2 gpurun_out/${T}_pytest_gpu.txt
  timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
  OUT=gpurun_out/${T}_line bash tools/profile_line.sh || exit 1
  timeout -k 10 600 bash tools/gpu/import_prof.sh || exit 1
else
  OUT=gpurun_out/prof_${T} bash tools/profile_round.sh ${CONFIGS:-fixed32 csr fixed4096 fixed32_1g ralledata fixed32_index} || exit 1
fi
echo ${T}_PART${PART:-1}_OK
