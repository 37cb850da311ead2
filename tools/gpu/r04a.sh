#!/bin/bash
# Round 4, first GPU session: the GPU suite (new: CSR byte-shard tests, table-form fixes) and the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04a_pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/r04a_pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/r04a_pytest_gpu.txt
timeout -k 10 400 python bench.py > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || { tail -20 gpurun_out/r04a_bench.err; exit 1; }
python - <<'P'
import json; d=json.load(open("gpurun_out/r04a_bench.json"))
print("headline", d["value"], d["roofline"]["frac"], d["verify"])
for k,v in d["secondary"].items():
    if k!="host": print(k, v.get("ms_per_step"), v.get("kernel_ms"), v["roofline"]["frac"], v.get("verify"))
P
echo R04A_OK
