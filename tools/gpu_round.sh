# One GPU call: parity tests, smoke, headline bench (+CPU baseline, phase
# timings on stderr), rocprofv3 kernel-trace summary of the bench, and the two
# PMC passes (FETCH_SIZE, WRITE_SIZE) of its query-eval kernel.  Optional A/B
# benches of the host walk variants when AB=1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
NKM_PROFILE=1 timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o trace --output-format csv -- $B > gpurun_out/bench_trace.json 2> gpurun_out/bench_trace.err && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o fetch --output-format csv -- $B > gpurun_out/pmc_fetch.json 2> gpurun_out/pmc_fetch.err && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o write --output-format csv -- $B > gpurun_out/pmc_write.json 2> gpurun_out/pmc_write.err
rc=$?
if [ $rc -eq 0 ] && [ "${AB:-0}" = "1" ]; then
  for v in "NKM_FAST=0" "NKM_DENSE=0" "NKM_FAST=1"; do
    env $v NKM_PROFILE=1 timeout -k 10 300 python bench.py --steps 7 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { rc=$?; break; }
  done
fi
echo EXIT $rc
