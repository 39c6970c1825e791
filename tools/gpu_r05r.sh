# Round 5: walk rewrites (DenseRun::fast_step, ReplayCore::fast_row: locals,
# batched output): PMU A/B against the round's earlier build on the box host,
# the walk / packed / range parity tests, then C3, C5 and C2 lines.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05r}
{
for b in replay_bench_r05old replay_bench; do
  echo "== $b"
  RB_MODE=c3 RB_PERF=1 timeout -k 10 120 tools/$b 1000000 20 0
  RB_MODE=c5 timeout -k 10 120 tools/$b 1000000 10 0
  RB_MODE=c5 RB_SHUFFLE=1 timeout -k 10 120 tools/$b 1000000 5 0
done
} > gpurun_out/${T}_walk_perf.txt 2>&1
grep -E "perf|c5" gpurun_out/${T}_walk_perf.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "c3 or c4 or c5 or exact_walk or pipelined or trim or packed or pool_runs or range or mixed or session or override" > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error|assert" gpurun_out/${T}_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for k in 3a 5a 2a 3b; do
  C=${k:0:1}
  NKM_PROFILE=2 timeout -k 10 300 python bench.py --config $C --steps 10 --no-cpu-baseline > gpurun_out/${T}_c$k.json 2> gpurun_out/${T}_c$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c$k.json').read().strip().splitlines()[-1])
print('c$k', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), 'ms_per_step', round(d['ms_per_step'], 2))"
  grep -E "pool walks|pool runs|batch 1 \(range\)" gpurun_out/${T}_c$k.err | tail -2 | sed 's/.*sum: //; s/gather+reset.*last/last/; s/.*merges | //'
done
