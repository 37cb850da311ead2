#!/bin/bash
# Round 4: the whole GPU suite, the import A/B (head-key isolation probes), the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/r04j
mkdir -p $O
P=k2hash_amd/lib/probe
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 300 python3 tools/import_step.py --ab $P/nohead.so,$P/nosearch.so,$P/nosort.so,$P/head.so --rounds 7 --calls 10 2>&1 | grep -v Warn | cut -c1-110
for lib in tree nohead head; do
  arg=""; [ $lib != tree ] && arg=$R/$P/$lib.so
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$lib -o run -- python3 $R/tools/import_probe.py $arg > $O/$lib.log 2>&1) || { tail $O/$lib.log; exit 1; }
  echo "== $lib"; python3 tools/kernel_trace_table.py $O/$lib/run_kernel_trace.csv "tsv_" 10 | cut -c1-100
done
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 - <<'P'
import json; d=json.load(open("gpurun_out/r04j/bench.json"))
print("headline", d["value"], d["roofline"]["frac"], d["verify"])
for k,v in d["secondary"].items():
    if k!="host": print(k, v.get("ms_per_step"), v.get("kernel_ms"), v["roofline"]["frac"], v.get("verify"))
P
echo R04J_IMPORT_BENCH_OK
timeout -k 10 300 python3 tools/ab_libs.py --libs k2hash_amd/lib/probe/csr_pf.so --config csr --rounds 5 --reps 10 2>&1 | grep -v Warn | cut -c1-160
echo R04J_CSR_OK
