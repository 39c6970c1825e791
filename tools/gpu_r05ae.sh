# Round 5: flat posting-list directory, three-sweep contiguous pool plan for
# packed batches, assembly count sweep without per-row MaxCount reads —
# parity (GPU parity + full-size digests + delivery), then C5 with
# NKM_PRUNS=1/0 interleaved and C3 x2.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05ae}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_full_size_golden.py tests/test_delivery.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error|assert" gpurun_out/${T}_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
line() {
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), 'ms_per_step', round(d['ms_per_step'], 2))" $1 "$2"
}
for k in a b c; do
  for m in 1 0; do
    NKM_PRUNS=$m NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 5 --steps 10 --no-cpu-baseline > gpurun_out/${T}_c5_${m}$k.json 2> gpurun_out/${T}_c5_${m}$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c5_${m}$k.err; exit 1; }
    line gpurun_out/${T}_c5_${m}$k.json "c5 pruns=$m $k"
    grep -E "plan_pools" gpurun_out/${T}_c5_${m}$k.err | tail -2
    grep -oE "assemble [0-9.]+, search [0-9.]+" gpurun_out/${T}_c5_${m}$k.err | tail -3 | tr '\n' ' '; echo
  done
done
for k in a b; do
  NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 3 --steps 10 --no-cpu-baseline > gpurun_out/${T}_c3_$k.json 2> gpurun_out/${T}_c3_$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c3_$k.err; exit 1; }
  line gpurun_out/${T}_c3_$k.json "c3 $k"
done
