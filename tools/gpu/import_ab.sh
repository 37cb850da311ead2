#!/bin/bash
# Same-process A/B of the k2himport scan: the tree's library against other builds (probe
# libraries from tools/probe_build.py), after the import GPU tests; then the tree's per-kernel
# times (rocprofv3 kernel trace of tools/import_probe.py) and PMC counters per kernel.
#   gpurun -- 'OUT=r04y LIBS=k2hash_amd/lib/probe/prev.so bash tools/gpu/import_ab.sh'
#   (NOPARITY=1: time probe libraries whose results are wrong by design)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/${OUT:-import_ab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_import.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
[ -n "$LIBS" ] && { timeout -k 10 300 python3 tools/import_step.py --ab $LIBS ${NOPARITY:+--no-parity} --rounds 7 --calls 10 2>&1 | grep -v Warn || exit 1; }
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tree -o run -- python3 $R/tools/import_probe.py > $O/tree.log 2>&1) || { tail $O/tree.log; exit 1; }
python3 tools/kernel_trace_table.py $O/tree/run_kernel_trace.csv "tsv_" 10 | cut -c1-100
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "tsv_" --output-format csv -d $O/pmc$i -o pmc -- python3 $R/tools/import_step.py --calls 4 > $O/pmc$i.log 2>&1) || { tail $O/pmc$i.log; exit 1; }
done
python3 tools/kernel_pmc_table.py "tsv_" $O/pmc1 $O/pmc2 $O/pmc3 2>&1 | cut -c1-140
echo IMPORT_AB_OK
