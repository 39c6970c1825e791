# Round 5: the packed plan declines interleaved pools from a 2048-row prefix
# (C2's range batches no longer pay two sweeps for it) — GPU tests for the
# packed / range paths, then C2 x2 and C5 with the plan split.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05at}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_full_size_golden.py -m gpu -k "two_runs or pool_runs or range or c2 or c5 or packed" > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error|assert" gpurun_out/${T}_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for k in a b; do
  NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 2 --steps 10 --no-cpu-baseline > gpurun_out/${T}_c2_$k.json 2> gpurun_out/${T}_c2_$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c2_$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c2_$k.json').read().strip().splitlines()[-1])
print('c2 $k', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2))"
  grep -oE "plan [0-9.]+ \(rows [0-9.]+ pools [0-9.]+" gpurun_out/${T}_c2_$k.err | tail -3 | tr '\n' ' '; echo
done
NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 5 --steps 8 --no-cpu-baseline > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c5.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c5.json').read().strip().splitlines()[-1])
print('c5', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2))"
grep -E "3 sweeps" gpurun_out/${T}_c5.err | tail -2
