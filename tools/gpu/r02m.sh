#!/bin/bash
# RALLEDATA gather kernel profile (trace + PMC), then the default bench line
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/prof_r02m bash tools/profile_round.sh ralledata
timeout -k 10 600 python -u bench.py > gpurun_out/r02m_bench.json 2> gpurun_out/r02m_bench.err
python3 -c "
import json; d=json.load(open('gpurun_out/r02m_bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('valu_frac'))
for k,v in d.get('secondary',{}).items(): print(k, {kk: v.get(kk) for kk in ('value','kernel_ms','verify')}, (v.get('roofline') or {}).get('frac'))
"
