#!/bin/bash
# Round 4: the entry-state scan with tiles of 1024 / 2048 blocks (probe/tile8.so, tile16.so) vs 512
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/r04zd
mkdir -p $O
P=k2hash_amd/lib/probe
timeout -k 10 300 python3 tools/import_step.py --ab $P/prev.so,$P/tile8.so,$P/tile16.so --rounds 7 --calls 10 2>&1 | grep -v Warn | cut -c1-110
for lib in tile8 tile16; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$lib -o run -- python3 $R/tools/import_probe.py $R/$P/$lib.so > $O/$lib.log 2>&1) || { tail $O/$lib.log; exit 1; }
  echo "== $lib"; python3 tools/kernel_trace_table.py $O/$lib/run_kernel_trace.csv "tsv_" 10 | cut -c1-100
done
echo R04ZD_OK
