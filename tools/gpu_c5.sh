# GPU call for the RevPrecision work: the packed / rev parity tests first,
# then every -m gpu test, then the C5 bench (phases), C5 + override, the C3
# headline, and a kernel-trace profile of C5.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-c5}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "packed or c5 or rev" --timeout 300 --timeout-method thread > gpurun_out/${T}_rev_tests.log 2>&1 || { echo REV_TESTS_FAIL; tail -40 gpurun_out/${T}_rev_tests.log; exit 1; }
tail -1 gpurun_out/${T}_rev_tests.log
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 5 --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.err || { echo C5_FAIL; tail -20 gpurun_out/${T}_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_c5.json'));r=d['roofline'];print('C5',d['value']/1e6,d['p50_ms'],r['kernel'],r['avg_launch_ms'],r['frac'])"
NKM_PROFILE=1 timeout -k 10 300 python bench.py --config 5 --override --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c5o.json 2> gpurun_out/${T}_c5o.err || { echo C5O_FAIL; tail -20 gpurun_out/${T}_c5o.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_c5o.json'));r=d['roofline'];print('C5o',d['value']/1e6,d['p50_ms'],r['kernel'],r['avg_launch_ms'],r['frac'])"
NKM_PROFILE=2 timeout -k 10 300 python bench.py --steps 11 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.err || { echo C3_FAIL; tail -20 gpurun_out/${T}_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_c3.json'));r=d['roofline'];print('C3',d['value']/1e6,d['p50_ms'],r['kernel'],r['avg_launch_ms'],r['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof5 -o run -- python3 bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_prof5.log 2>&1 || { echo PROF5_FAIL; tail -20 gpurun_out/${T}_prof5.log; exit 1; }
head -8 gpurun_out/${T}_prof5/run_kernel_stats.csv
