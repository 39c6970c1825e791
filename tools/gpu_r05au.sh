# Round 5: a signature's single MUST term kept inline (source_of reads no term
# list) — GPU tests for the packed / processCustom / C5 paths, then C5
# against HEAD (ab/libnakama_mm_head.so), interleaved x3.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05au}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_full_size_golden.py -m gpu -k "c5 or packed or pool or custom or rev or two_runs or c1 or c2" > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error|assert" gpurun_out/${T}_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
line() {
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), 'ms_per_step', round(d['ms_per_step'], 2))" $1 "$2"
}
HEAD_SO=$GRAFT_REPO_ROOT/ab/libnakama_mm_head.so
for k in a b c; do
  for v in new head; do
    if [ $v = head ]; then L=$HEAD_SO; else L=; fi
    NKM_LIBRARY=$L NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 5 --steps 10 --no-cpu-baseline > gpurun_out/${T}_c5_$v$k.json 2> gpurun_out/${T}_c5_$v$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c5_$v$k.err; exit 1; }
    line gpurun_out/${T}_c5_$v$k.json "c5 $v $k"
    grep -oE "assemble_packed: [0-9]+ rows \| sources [0-9.]+" gpurun_out/${T}_c5_$v$k.err | tail -3 | tr '\n' ' '; echo
  done
done
