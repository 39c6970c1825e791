# Quick GPU call for host-path work on C3: the full-size C3 digests (every
# host path), the small parity tests of the parallel replay, then the headline
# bench with per-phase timings (NKM_PROFILE=1 on stderr).  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-c3}
timeout -k 10 600 python -u -m pytest tests/test_full_size_golden.py tests/test_gpu_parity.py -x -v -m gpu -k "c3 or pipelined or parallel or exact_walk or c4" --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/${T}_tests.log; exit 1; }
NKM_PROFILE=1 timeout -k 10 300 python bench.py --steps 11 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_bench.err; exit 1; }
tail -2 gpurun_out/${T}_tests.log
cat gpurun_out/${T}_bench.json
