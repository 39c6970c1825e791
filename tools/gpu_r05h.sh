# Round 5: C3 A/B — pipelined-merge chunks per worker (NKM_MCH) and the
# workers' pre-wake after each job (NKM_PREWAKE) — with phase profiles.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05h}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "pipelined_merge or c3_parties or pool_runs" > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error|assert" gpurun_out/${T}_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for V in "2 0" "2 1" "8 1" "16 1" "2 0" "2 1" "8 1"; do
  set -- $V
  N=m$1_w$2
  NKM_MCH=$1 NKM_PREWAKE=$2 NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 3 --steps 8 --no-cpu-baseline > gpurun_out/${T}_c3_$N.json 2> gpurun_out/${T}_c3_$N.err || { echo BENCH_FAIL $N; tail -20 gpurun_out/${T}_c3_$N.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c3_$N.json').read().strip().splitlines()[-1])
print('$N', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), 'ms_per_step', round(d['ms_per_step'], 2))"
  grep -E "pool walks" gpurun_out/${T}_c3_$N.err | tail -2 | sed 's/.*gather beside//'
  grep -E "finish: retire" gpurun_out/${T}_c3_$N.err | tail -2
done
