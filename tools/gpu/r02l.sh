#!/bin/bash
# clock probe (fixed32, 4 KiB, CSR), the full GPU suite, the default bench line
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/clock_probe.py --json gpurun_out/clock_probe.json
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02l_pytest.txt 2>&1 || { tail -30 gpurun_out/r02l_pytest.txt; exit 1; }
tail -2 gpurun_out/r02l_pytest.txt
timeout -k 10 600 python -u bench.py > gpurun_out/r02l_bench.json 2> gpurun_out/r02l_bench.err
python3 -c "
import json; d=json.load(open('gpurun_out/r02l_bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('valu_frac'))
for k,v in d.get('secondary',{}).items(): print(k, {kk: v.get(kk) for kk in ('value','kernel_ms','ms_per_step')}, (v.get('roofline') or {}).get('frac'))
"
