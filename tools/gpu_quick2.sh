# Quick GPU check: a -k selection of the -m gpu tests ($2), then the C5 and
# C3 benches with phase timings.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-q}
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "${2:-packed or c5 or c3 or c4}" --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 5 --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.err || { echo C5_FAIL; tail -20 gpurun_out/${T}_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_c5.json'));r=d['roofline'];print('C5',d['value']/1e6,d['p50_ms'],r['kernel'],r['avg_launch_ms'],r['frac'])"
grep "plan_pools\|packed" gpurun_out/${T}_c5.err | tail -4
NKM_PROFILE=1 timeout -k 10 300 python bench.py --steps 11 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.err || { echo C3_FAIL; tail -20 gpurun_out/${T}_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_c3.json'));r=d['roofline'];print('C3',d['value']/1e6,d['p50_ms'],r['kernel'],r['avg_launch_ms'],r['frac'])"
