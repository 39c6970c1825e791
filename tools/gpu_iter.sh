# Iteration GPU call: every -m gpu test (or the -k selection in $2), then
# the C3 headline bench and the C4 bench with phase timings.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-it}
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -k "$K" --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
fi
tail -1 gpurun_out/${T}_gpu_tests.log
NKM_PROFILE=2 timeout -k 10 300 python bench.py --steps 11 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_bench.json'));r=d['roofline'];print('C3',d['value']/1e6,d['p50_ms'],r['kernel'],r['avg_launch_ms'],r['frac'])"
NKM_PROFILE=1 timeout -k 10 300 python bench.py --config 4 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c4.json 2> gpurun_out/${T}_c4.err || { echo BENCH4_FAIL; tail -20 gpurun_out/${T}_c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_c4.json'));r=d['roofline'];print('C4',d['value']/1e6,d['p50_ms'],r['kernel'],r['avg_launch_ms'],r['frac'])"
