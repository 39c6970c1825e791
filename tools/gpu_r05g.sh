# Round 5: replay_runs (C5's run-ordered pool replay) — its parity tests, the
# full-size C5 digests, then the C5 line with phase profiles.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05g}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_full_size_golden.py -m gpu -k "pool_runs or packed_rev or c5" > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error|assert" gpurun_out/${T}_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c5.err; exit 1; }
NKM_RUNS=0 NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > gpurun_out/${T}_c5_runs0.json 2> gpurun_out/${T}_c5_runs0.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c5_runs0.err; exit 1; }
for f in c5 c5_runs0; do
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_$f.json').read().strip().splitlines()[-1])
print('$f', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), 'ms_per_step', round(d['ms_per_step'], 2))"
done
grep -E "pool runs|pass [0-9.]+ ms" gpurun_out/${T}_c5.err | tail -6
