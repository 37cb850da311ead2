#!/bin/bash
# round 3: import tests + profile after the batched TSV stage loads; RALLEDATA lab A/B,
# variant 7 (record offsets of every segment loaded without branches); CSR variants 9/10 again
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_import.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03v_pytest_import.txt 2>&1
tail -2 gpurun_out/r03v_pytest_import.txt
timeout -k 10 600 bash tools/gpu/r03_import_prof.sh
timeout -k 10 300 python tools/import_step.py --calls 20 > gpurun_out/r03v_import_step.txt 2>&1
tail -1 gpurun_out/r03v_import_step.txt
timeout -k 10 240 python tools/lab_ab.py ralle --variants 0 7 --reps 9 > gpurun_out/r03v_ralle_ab.json 2> gpurun_out/r03v_ralle_ab.err
cat gpurun_out/r03v_ralle_ab.json
timeout -k 10 300 python tools/lab_ab.py csr --variants 0 9 10 --reps 7 > gpurun_out/r03v_csr_ab.json 2> gpurun_out/r03v_csr_ab.err
cat gpurun_out/r03v_csr_ab.json
echo R03V_OK
