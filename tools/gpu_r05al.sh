# Round 5: replay_runs outputs before its byte stores, finish retire with base
# pointers in locals — GPU parity subset, then C5 and C3 against HEAD.
#
#
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05al}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_full_size_golden.py -m gpu -k "c3 or c5 or mixed or pool or delivery or custom" > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error|assert" gpurun_out/${T}_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
line() {
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), 'ms_per_step', round(d['ms_per_step'], 2))" $1 "$2"
}
HEAD_SO=$GRAFT_REPO_ROOT/ab/libnakama_mm_head.so
for cfg in 5 3; do
  for k in a b; do
    for v in new head; do
      if [ $v = head ]; then L=$HEAD_SO; else L=; fi
      NKM_LIBRARY=$L NKM_PROFILE=2 timeout -k 10 300 python bench.py --config $cfg --steps 8 --no-cpu-baseline > gpurun_out/${T}_c${cfg}_$v$k.json 2> gpurun_out/${T}_c${cfg}_$v$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c${cfg}_$v$k.err; exit 1; }
      line gpurun_out/${T}_c${cfg}_$v$k.json "c$cfg $v $k"
      grep -oE "replay: gather [0-9.]+ job [0-9.]+" gpurun_out/${T}_c${cfg}_$v$k.err | tail -3 | tr '\n' ' '; echo
      grep -oE "pool runs: .*|finish: retire [0-9.]+" gpurun_out/${T}_c${cfg}_$v$k.err | tail -4 | cut -c1-140 | tr '\n' ' '; echo
    done
  done
done
