# Round 5: range batches with the leaves gathered in the tiers' job; expired
# lists uninitialised.  Range / C2 / trim tests, full-size C2 + C3 digests,
# then C2 x3 and C3 x1 with phase profiles.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05j}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_full_size_golden.py -m gpu -k "range or c2 or trim or mixed or full_size_pass" > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error|assert" gpurun_out/${T}_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for k in 2a 2b 2c 3a; do
  C=${k:0:1}
  NKM_PROFILE=2 timeout -k 10 300 python bench.py --config $C --steps 8 --no-cpu-baseline > gpurun_out/${T}_c$k.json 2> gpurun_out/${T}_c$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c$k.json').read().strip().splitlines()[-1])
print('c$k', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), 'ms_per_step', round(d['ms_per_step'], 2))"
  grep -E "batch 1 \(range\)|pool walks" gpurun_out/${T}_c$k.err | tail -2 | sed 's/.*merges | //; s/.*sum: //'
done
