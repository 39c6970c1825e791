# GPU parity tests, then the host-thread sweep of the C3 pass (NKM_PROFILE phases).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS FAILED; exit 1; }
for t in ${NKM_SWEEP:-1 8 16}; do
  NKM_THREADS=$t NKM_PROFILE=1 timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/bench_t$t.json 2> gpurun_out/bench_t$t.err || exit 1
done
echo EXIT $?
