#!/bin/bash
# Round 4: (import) pass-B records staged in LDS and written out coalesced; (RALLEDATA) the
# piece table built by waves 1-3 while wave 0 hashes.  Tests, same-process A/B against HEAD
# (probe/prev.so), PMC counters of the tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/r04y
mkdir -p $O
P=k2hash_amd/lib/probe
timeout -k 10 600 python -u -m pytest tests/test_import.py tests/test_ralledata.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 300 python3 tools/import_step.py --ab $P/prev.so --rounds 7 --calls 10 2>&1 | grep -v Warn | cut -c1-110
timeout -k 10 300 python3 tools/ab_libs.py --config ralledata --libs $P/prev.so 2>&1 | grep -v Warn | cut -c1-160
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tree -o run -- python3 $R/tools/import_probe.py > $O/tree.log 2>&1) || { tail $O/tree.log; exit 1; }
python3 tools/kernel_trace_table.py $O/tree/run_kernel_trace.csv "tsv_" 10 | cut -c1-100
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "tsv_" --output-format csv -d $O/pmc$i -o pmc -- python3 $R/tools/import_step.py --calls 4 > $O/pmc$i.log 2>&1) || { tail $O/pmc$i.log; exit 1; }
done
python3 tools/kernel_pmc_table.py "tsv_" $O/pmc1 $O/pmc2 $O/pmc3 2>&1 | cut -c1-140
(cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-include-regex "ralledata" --output-format csv -d $O/rpmc -o pmc -- python3 $R/bench.py --config ralledata --steps 5 --warmup 2 > $O/rpmc.log 2>&1) || { tail $O/rpmc.log; exit 1; }
python3 tools/kernel_pmc_table.py "ralledata" $O/rpmc 2>&1 | cut -c1-140
echo R04Y_OK
