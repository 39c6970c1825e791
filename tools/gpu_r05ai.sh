# Round 5: the pipelined merge's output streams written non-temporally
# (NKM_MNT=1) against plain stores — parity with NKM_MNT=1 (C3 / C4 / mixed /
# pools / delivery), then C4 and C3 interleaved MNT=0/1.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05ai}
NKM_MNT=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_full_size_golden.py tests/test_delivery.py -m gpu -k "c3 or c4 or mixed or pool or delivery" > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error|assert" gpurun_out/${T}_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
line() {
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), 'ms_per_step', round(d['ms_per_step'], 2))" $1 "$2"
}
for cfg in 4 3; do
  for k in a b; do
    for m in 1 0; do
      NKM_MNT=$m NKM_PROFILE=2 timeout -k 10 300 python bench.py --config $cfg --steps 8 --no-cpu-baseline > gpurun_out/${T}_c${cfg}_m$m$k.json 2> gpurun_out/${T}_c${cfg}_m$m$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c${cfg}_m$m$k.err; exit 1; }
      line gpurun_out/${T}_c${cfg}_m$m$k.json "c$cfg mnt=$m $k"
      grep -oE "last walk ends [0-9.]+, job [0-9.]+ ms \([0-9]+ merge chunks: sum [0-9.]+" gpurun_out/${T}_c${cfg}_m$m$k.err | tail -3 | tr '\n' ' '; echo
      grep -oE "finish [0-9.]+ ms" gpurun_out/${T}_c${cfg}_m$m$k.err | tail -3 | tr '\n' ' '; echo
    done
  done
done
