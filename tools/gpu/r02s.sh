#!/bin/bash
# round-2 final: GPU suite, profile round (trace + PMC) of every config, default bench line
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02s_pytest.txt 2>&1 || { tail -30 gpurun_out/r02s_pytest.txt; exit 1; }
tail -2 gpurun_out/r02s_pytest.txt
OUT=gpurun_out/prof_r02s bash tools/profile_round.sh fixed32 csr fixed4096 fixed32_1g ralledata
timeout -k 10 600 python -u bench.py > gpurun_out/r02s_bench.json 2> gpurun_out/r02s_bench.err
python3 -c "
import json; d=json.load(open('gpurun_out/r02s_bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('valu_frac'))
for k,v in d.get('secondary',{}).items(): print(k, {kk: v.get(kk) for kk in ('value','kernel_ms','verify')}, (v.get('roofline') or {}).get('frac'))
print(d['cpu_baseline']['value'], d['cpu_baseline']['cores'])
"
