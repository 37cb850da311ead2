set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02a_smoke.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/r02a_bench.json 2> gpurun_out/r02a_bench.err
timeout -k 10 300 python -u bench.py --config csr --no-cpu-baseline > gpurun_out/r02a_bench_csr.json 2>>gpurun_out/r02a_bench.err
timeout -k 10 300 python -u bench.py --config fixed4096 --no-cpu-baseline > gpurun_out/r02a_bench_4k.json 2>>gpurun_out/r02a_bench.err
cat gpurun_out/r02a_*.json
