#!/bin/bash
# Extra bench lines of the widened rows (bucket index, h2, RALLEDATA) + host-path rate.
set -o pipefail
OUT=${OUT:-gpurun_out/extra}
mkdir -p "$OUT"
for a in "--index" "--second" "--config csr --index" "--config fixed4096 --index" "--config ralledata"; do
  name=$(echo $a | tr -d ' -')
  timeout -k 10 200 python3 bench.py $a --no-cpu-baseline > "$OUT/bench_$name.json" 2>/dev/null || { echo "bench $a failed"; exit 1; }
done
timeout -k 10 200 python3 tools/host_rate.py > "$OUT/host_rate.json" 2> "$OUT/host_rate.err" || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/$OUT/prof_ralledata" -o run -- python3 "$OLDPWD/bench.py" --config ralledata --steps 10 --warmup 3 --no-cpu-baseline > "$OLDPWD/$OUT/prof_ralledata.log" 2>&1) || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/$OUT/prof_index" -o run -- python3 "$OLDPWD/bench.py" --index --steps 10 --warmup 3 --no-cpu-baseline > "$OLDPWD/$OUT/prof_index.log" 2>&1) || exit 1
echo EXTRA_OK
