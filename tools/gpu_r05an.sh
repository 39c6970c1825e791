# Round 5: the packed-plan test with buckets in two runs, then the default C3
# line three times (box-to-box / run-to-run spread of the headline).  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05an}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "two_runs or pool_runs" > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAILED|Error|assert" gpurun_out/${T}_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for k in a b c; do
  timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/${T}_c3_$k.json 2> gpurun_out/${T}_c3_$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c3_$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c3_$k.json').read().strip().splitlines()[-1])
print('c3 $k', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2))"
done
