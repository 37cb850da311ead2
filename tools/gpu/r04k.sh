#!/bin/bash
# Round 4: import -- the entry-state scan over pass-A blocks again (per-unit prefixes derived), tests + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/r04k
mkdir -p $O
P=k2hash_amd/lib/probe
timeout -k 10 600 python -u -m pytest tests/test_import.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_import.txt 2>&1 || { tail -40 $O/pytest_import.txt; exit 1; }
tail -1 $O/pytest_import.txt
timeout -k 10 300 python3 tools/import_step.py --ab $P/prev.so,$P/head.so --rounds 7 --calls 10 2>&1 | grep -v Warn | cut -c1-110
for lib in tree prev; do
  arg=""; [ $lib != tree ] && arg=$R/$P/$lib.so
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$lib -o run -- python3 $R/tools/import_probe.py $arg > $O/$lib.log 2>&1) || { tail $O/$lib.log; exit 1; }
  echo "== $lib"; python3 tools/kernel_trace_table.py $O/$lib/run_kernel_trace.csv "tsv_" 10 | cut -c1-100
done
echo R04K_OK
