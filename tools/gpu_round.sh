# One GPU call: parity tests, smoke, headline bench (+CPU baseline), rocprof
# kernel-trace summary and the two PMC passes (FETCH_SIZE, WRITE_SIZE).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o trace --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_trace.json 2> gpurun_out/bench_trace.err && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o fetch --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/bench_fetch.json 2> gpurun_out/bench_fetch.err && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o write --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/bench_write.json 2> gpurun_out/bench_write.err
echo EXIT $?
