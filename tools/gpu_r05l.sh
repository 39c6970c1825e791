# Round 5: C3 A/B of the pipelined merge's wait (NKM_MWAIT: sleep µs vs 0 =
# sched_yield), interleaved, plus the C5 line after the u8 pack positions.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05l}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "pipelined_merge or c3_parties" > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error|assert" gpurun_out/${T}_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for k in 0a 20a 0b 20b 0c 20c 50a; do
  W=${k%?}
  NKM_MWAIT=$W NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 3 --steps 10 --no-cpu-baseline > gpurun_out/${T}_c3_$k.json 2> gpurun_out/${T}_c3_$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c3_$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c3_$k.json').read().strip().splitlines()[-1])
print('mwait $k', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), 'ms_per_step', round(d['ms_per_step'], 2))"
  grep -E "pool walks" gpurun_out/${T}_c3_$k.err | tail -3 | sed 's/.*sum: //; s/gather+reset.*last/last/'
done
