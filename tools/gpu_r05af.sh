# Round 5: gather without DenseCold, block-scrambled posting directory —
# every GPU test, then C5 and C3 interleaved against the previous commit's
# library (ab/libnakama_mm_head.so through NKM_LIBRARY); C4 with the
# gather's non-temporal stores off / on (NKM_GNT).  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05af}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error|assert" gpurun_out/${T}_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
NKM_GNT=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_full_size_golden.py -m gpu -k "c3 or c4 or mixed or pool" > gpurun_out/${T}_tests_gnt.log 2>&1 || { echo TESTS_GNT_FAIL; grep -E "^FAILED|Error|assert" gpurun_out/${T}_tests_gnt.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_tests_gnt.log
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
      NKM_LIBRARY=$L NKM_PROFILE=1 timeout -k 10 300 python bench.py --config $cfg --steps 10 --no-cpu-baseline > gpurun_out/${T}_c${cfg}_$v$k.json 2> gpurun_out/${T}_c${cfg}_$v$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c${cfg}_$v$k.err; exit 1; }
      line gpurun_out/${T}_c${cfg}_$v$k.json "c$cfg $v $k"
      grep -oE "assemble [0-9.]+, search [0-9.]+ ms \[kernel [0-9.]+ ms\], replay [0-9.]+" gpurun_out/${T}_c${cfg}_$v$k.err | tail -3 | tr '\n' ' '; echo
      grep -oE "replay: gather [0-9.]+ job [0-9.]+" gpurun_out/${T}_c${cfg}_$v$k.err | tail -3 | tr '\n' ' '; echo
    done
  done
done
for k in a b; do
  for g in 0 1; do
    NKM_GNT=$g NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 4 --steps 8 --no-cpu-baseline > gpurun_out/${T}_c4_g$g$k.json 2> gpurun_out/${T}_c4_g$g$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c4_g$g$k.err; exit 1; }
    line gpurun_out/${T}_c4_g$g$k.json "c4 gnt=$g $k"
    grep -oE "replay: gather [0-9.]+ job [0-9.]+" gpurun_out/${T}_c4_g$g$k.err | tail -3 | tr '\n' ' '; echo
    grep -oE "last walk ends [0-9.]+, job [0-9.]+ ms" gpurun_out/${T}_c4_g$g$k.err | tail -2 | tr '\n' ' '; echo
  done
done
