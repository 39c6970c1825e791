# Round 5: dense-pool gather task size (NKM_GTASK: list positions per task
# over all pools; 16384 default) — parity at 4096, then C3 and C4 with 16384 /
# 4096 / 8192 interleaved.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05ap}
NKM_GTASK=4096 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_full_size_golden.py -m gpu -k "c3 or c4 or mixed or pool" > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error|assert" gpurun_out/${T}_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
line() {
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), 'ms_per_step', round(d['ms_per_step'], 2))" $1 "$2"
}
for cfg in 3 4; do
  for k in a b; do
    for g in 16384 4096 8192; do
      NKM_GTASK=$g NKM_PROFILE=2 timeout -k 10 300 python bench.py --config $cfg --steps 10 --no-cpu-baseline > gpurun_out/${T}_c${cfg}_g$g$k.json 2> gpurun_out/${T}_c${cfg}_g$g$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c${cfg}_g$g$k.err; exit 1; }
      line gpurun_out/${T}_c${cfg}_g$g$k.json "c$cfg gtask=$g $k"
      grep -oE "walks [0-9.]+ \(max [0-9.]+\)|last walk ends [0-9.]+, job [0-9.]+|gather [0-9.]+, bounds" gpurun_out/${T}_c${cfg}_g$g$k.err | tail -6 | tr '\n' ' '; echo
    done
  done
done
