# Round 5: assembly count sweep without per-row MaxCount reads — C3 / C4 /
# mixed parity and full-size digests, then C3 x3 with the count-sweep profile.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05ad}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_full_size_golden.py -m gpu -k "c3 or c4 or mixed or c1_pool or top_tier or range" > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error|assert" gpurun_out/${T}_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for k in a b c; do
  NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 3 --steps 10 --no-cpu-baseline > gpurun_out/${T}_c3_$k.json 2> gpurun_out/${T}_c3_$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c3_$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c3_$k.json').read().strip().splitlines()[-1])
print('c3 $k', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), 'ms_per_step', round(d['ms_per_step'], 2))"
  grep -E "count sweep|asm: count" gpurun_out/${T}_c3_$k.err | tail -2 | sed 's/.*prologue/prologue/'
done
