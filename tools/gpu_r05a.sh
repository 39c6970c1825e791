# Round 5, first GPU call: the -m gpu parity tests (new: CountMultiple trim
# scenarios, configs 17/18, bulk Insert id-field fallback), smoke, the C3 line
# and a profiled C5 + override line.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05a}
timeout -k 10 900 python -u -m pytest -q --timeout 400 --timeout-method thread tests -m gpu > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
NKM_PROFILE=1 timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_bench.err; exit 1; }
NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 5 --override --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c5o.json 2> gpurun_out/${T}_c5o.err || { echo BENCH_FAIL c5o; tail -20 gpurun_out/${T}_c5o.err; exit 1; }
tail -c 600 gpurun_out/${T}_bench.json; echo; tail -c 900 gpurun_out/${T}_c5o.json
