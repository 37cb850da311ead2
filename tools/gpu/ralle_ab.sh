#!/bin/bash
# Same-process A/B of the RALLEDATA kernel: the tree's library against other builds, after
# the RALLEDATA GPU tests; then the tree's PMC counters over bench.py --config ralledata.
#   gpurun -- 'OUT=r04za LIBS=k2hash_amd/lib/probe/prev.so bash tools/gpu/ralle_ab.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/${OUT:-ralle_ab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ralledata.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
[ -n "$LIBS" ] && { timeout -k 10 300 python3 tools/ab_libs.py --config ralledata --libs $LIBS 2>&1 | grep -v Warn | cut -c1-160 || exit 1; }
(cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex "ralledata" --output-format csv -d $O/rpmc -o pmc -- python3 $R/bench.py --config ralledata --steps 5 --warmup 2 > $O/rpmc.log 2>&1) || { tail $O/rpmc.log; exit 1; }
python3 tools/kernel_pmc_table.py "ralledata" $O/rpmc 2>&1 | cut -c1-140
echo RALLE_AB_OK
