# Round 5: gather task size chosen by where the gather runs (4096 beside the
# walks, 16384 before them) — GPU parity subset, then C3 auto / 2048 / 16384
# interleaved and C4 auto.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05aq}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_full_size_golden.py tests/test_delivery.py -m gpu -k "c3 or c4 or mixed or pool or delivery" > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error|assert" gpurun_out/${T}_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
line() {
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), 'ms_per_step', round(d['ms_per_step'], 2))" $1 "$2"
}
for k in a b c; do
  for g in auto 2048 16384; do
    if [ $g = auto ]; then G=; else G=$g; fi
    NKM_GTASK=$G NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 3 --steps 10 --no-cpu-baseline > gpurun_out/${T}_c3_g$g$k.json 2> gpurun_out/${T}_c3_g$g$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c3_g$g$k.err; exit 1; }
    line gpurun_out/${T}_c3_g$g$k.json "c3 gtask=$g $k"
    grep -oE "walks [0-9.]+ \(max [0-9.]+\)|last walk ends [0-9.]+, job [0-9.]+" gpurun_out/${T}_c3_g$g$k.err | tail -4 | tr '\n' ' '; echo
  done
done
NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 4 --steps 8 --no-cpu-baseline > gpurun_out/${T}_c4.json 2> gpurun_out/${T}_c4.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c4.err; exit 1; }
line gpurun_out/${T}_c4.json "c4 auto"
grep -oE "gather [0-9.]+, bounds" gpurun_out/${T}_c4.err | tail -2 | tr '\n' ' '; echo
