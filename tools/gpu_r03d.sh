# Round-3 re-entry GPU call: every -m gpu test on the current tree (hashed
# mscan included), smoke, the C3 headline bench and the C4 bench with phase
# timings, kernel-trace stats of both.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r03d}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
NKM_PROFILE=1 timeout -k 10 300 python bench.py --steps 11 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
NKM_PROFILE=1 timeout -k 10 300 python bench.py --config 4 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c4.json 2> gpurun_out/${T}_c4.err || { echo BENCH4_FAIL; tail -20 gpurun_out/${T}_c4.err; exit 1; }
cat gpurun_out/${T}_c4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof3 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_prof3.log 2>&1 || { echo PROF3_FAIL; tail -20 gpurun_out/${T}_prof3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof4 -o run -- python3 bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_prof4.log 2>&1 || { echo PROF4_FAIL; tail -20 gpurun_out/${T}_prof4.log; exit 1; }
echo DONE
