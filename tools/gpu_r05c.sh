# Round 5: the GPU tests, the hashed-scan study (tools/mhash_bench), then
# the C3, C4 and C5 + override lines with phase profiles and the C3 / C4
# kernel-trace summaries.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05e}
timeout -k 10 900 python -u -m pytest -q --timeout 400 --timeout-method thread tests -m gpu > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error" gpurun_out/${T}_gpu_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
timeout -k 10 120 tools/mhash_bench > gpurun_out/${T}_mhash_bench.txt 2>&1 || { echo MHB_FAIL; tail -20 gpurun_out/${T}_mhash_bench.txt; exit 1; }
grep -E "contig J4 grid.*dbg 0|lists WRONG" gpurun_out/${T}_mhash_bench.txt
NKM_PROFILE=1 timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_bench.err; exit 1; }
NKM_PROFILE=1 timeout -k 10 400 python bench.py --config 4 --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c4.json 2> gpurun_out/${T}_c4.err || { echo BENCH_FAIL c4; tail -20 gpurun_out/${T}_c4.err; exit 1; }
NKM_PROFILE=1 timeout -k 10 300 python bench.py --config 5 --override --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c5o.json 2> gpurun_out/${T}_c5o.err || { echo BENCH_FAIL c5o; tail -20 gpurun_out/${T}_c5o.err; exit 1; }
for f in bench c4 c5o; do
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_$f.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), r.get('kernel'), round(r['avg_launch_ms']*1e3, 2), 'us frac', round(r['frac'], 3), d['config'].get('override_step_ms'))"
done
for C in 3 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c${C}_prof -o run -- python3 bench.py --config $C --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c${C}_prof.log 2>&1 || { echo PROF_FAIL $C; tail -20 gpurun_out/${T}_c${C}_prof.log; exit 1; }
  head -6 gpurun_out/${T}_c${C}_prof/run_kernel_stats.csv
done
