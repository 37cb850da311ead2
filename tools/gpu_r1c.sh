#!/bin/bash
# bucket-index parity + GPU parity suite + fused-index bench + host rate
set -o pipefail
OUT=${OUT:-gpurun_out/r1c}
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?; tail -4 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit 1
for a in "" "--index" "--second" "--config csr --index" "--config fixed4096 --index"; do
  timeout -k 10 200 python3 bench.py $a --no-cpu-baseline > "$OUT/bench_$(echo $a | tr -d ' -').json" 2>/dev/null || exit 1
  cat "$OUT/bench_$(echo $a | tr -d ' -').json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['metric'][:60], round(d['value']/1e9,2),'G/s', round(d['kernel_ms']*1e3,1),'us', round(d['roofline']['frac'],3))"
done
timeout -k 10 200 python3 tools/host_rate.py > "$OUT/host_rate.json" 2> "$OUT/host_rate.err" && cat "$OUT/host_rate.json"
