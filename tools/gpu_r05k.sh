# Round 5: C2 A/B — range leaves gathered by each walker (NKM_RLEAF=0, with
# prefetch) vs across the workers (1), interleaved.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05k}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "range or c2 or pool_runs or packed_rev or c5_rev" > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error|assert" gpurun_out/${T}_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for k in 0a 1a 0b 1b 0c 1c; do
  L=${k:0:1}
  NKM_RLEAF=$L NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 2 --steps 10 --no-cpu-baseline > gpurun_out/${T}_c2_$k.json 2> gpurun_out/${T}_c2_$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c2_$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c2_$k.json').read().strip().splitlines()[-1])
print('rleaf $k', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), 'ms_per_step', round(d['ms_per_step'], 2))"
  grep -E "batch 1 \(range\)" gpurun_out/${T}_c2_$k.err | tail -2 | sed 's/.*merges | //'
done
NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.err || { echo BENCH_FAIL c5; tail -20 gpurun_out/${T}_c5.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c5.json').read().strip().splitlines()[-1])
print('c5', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), 'ms_per_step', round(d['ms_per_step'], 2))"
grep -E "plan_pools|pass [0-9.]+ ms" gpurun_out/${T}_c5.err | tail -2 | cut -c1-200
