# Round 5: processCustom candidates straight into the result arena (pinned
# chunks overlapped with the entry conversion): override tests, full-size
# C5 + override digests, then the C5o line with phases, NKM_CDIRECT=1 vs 0.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05aa}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_full_size_golden.py tests/test_delivery.py tests/test_multi.py -m gpu -k "custom or override or c5o" > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error|assert" gpurun_out/${T}_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for k in 1a 0a 1b; do
  D=${k:0:1}
  NKM_CDIRECT=$D NKM_PROFILE=2 timeout -k 10 400 python bench.py --config 5 --override --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c5o_$k.json 2> gpurun_out/${T}_c5o_$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c5o_$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c5o_$k.json').read().strip().splitlines()[-1])
print('cdirect $k', round(d['value']/1e6, 3), 'M/s p50', round(d['p50_ms'], 1), d['config'].get('override_step_ms'))"
  grep -E "custom enum|custom: sync" gpurun_out/${T}_c5o_$k.err | tail -2 | cut -c1-250
done
