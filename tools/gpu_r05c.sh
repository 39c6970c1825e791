# Round 5: the hashed-scan study (tools/gpu_mhash_study.sh), the GPU tests
# with the resident loop / counts-only scans on by default, then the C3, C4
# and C5 + override lines with phase profiles.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05c}
bash tools/gpu_mhash_study.sh $T || exit 1
timeout -k 10 900 python -u -m pytest -q --timeout 400 --timeout-method thread tests -m gpu > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error" gpurun_out/${T}_gpu_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
NKM_PROFILE=1 timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_bench.err; exit 1; }
NKM_PROFILE=1 timeout -k 10 400 python bench.py --config 4 --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c4.json 2> gpurun_out/${T}_c4.err || { echo BENCH_FAIL c4; tail -20 gpurun_out/${T}_c4.err; exit 1; }
NKM_PROFILE=1 timeout -k 10 300 python bench.py --config 5 --override --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c5o.json 2> gpurun_out/${T}_c5o.err || { echo BENCH_FAIL c5o; tail -20 gpurun_out/${T}_c5o.err; exit 1; }
for f in bench c4 c5o; do
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_$f.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), r.get('kernel'), round(r['avg_launch_ms']*1e3, 2), 'us frac', round(r['frac'], 3), d['config'].get('override_step_ms'))"
done
