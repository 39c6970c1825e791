# Round 5: the rewritten fast_step (locals, batched output) — its PMU counts on
# the box's host (replay_bench RB_PERF=1), walk parity tests, then C3 x2.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05q}
{
for b in replay_bench_r05old replay_bench replay_bench_r05old replay_bench; do
  echo "== $b"
  RB_MODE=c3 RB_PERF=1 timeout -k 10 120 tools/$b 1000000 20 0
  RB_MODE=c4 RB_PERF=1 timeout -k 10 120 tools/$b 4000000 10 0
  RB_MODE=c5 timeout -k 10 120 tools/$b 1000000 10 0
done
} > gpurun_out/${T}_walk_perf.txt 2>&1
cat gpurun_out/${T}_walk_perf.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_full_size_golden.py tests/test_replay_walks.py -m "gpu or not gpu" -k "c3 or c4 or exact_walk or pipelined or trim or walks" > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error|assert" gpurun_out/${T}_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for k in 3a 3b; do
  C=${k:0:1}
  NKM_PROFILE=2 timeout -k 10 300 python bench.py --config $C --steps 10 --no-cpu-baseline > gpurun_out/${T}_c$k.json 2> gpurun_out/${T}_c$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c$k.json').read().strip().splitlines()[-1])
print('c$k', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), 'ms_per_step', round(d['ms_per_step'], 2))"
  grep -E "pool walks" gpurun_out/${T}_c$k.err | tail -3 | sed 's/.*sum: //; s/gather+reset.*last/last/'
done
