# Round 5 final-tree run (after the prefix check and the inline MUST key): the
# whole GPU suite, smoke(), the default bench line, the C3 rocprofv3 summary,
# then the C4, C5, C2 and C5 + override lines.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05av}
timeout -k 10 1100 python -u -m pytest -q --timeout 400 --timeout-method thread tests -m gpu > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error" gpurun_out/${T}_gpu_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_bench.err; exit 1; }
tail -1 gpurun_out/${T}_bench.json | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c3_prof -o run -- python3 bench.py --config 3 --steps 10 --no-cpu-baseline > gpurun_out/${T}_c3_prof.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/${T}_c3_prof.log; exit 1; }
head -5 gpurun_out/${T}_c3_prof/run_kernel_stats.csv | cut -c1-160
for k in 4 5 2; do
  NKM_PROFILE=1 timeout -k 10 400 python bench.py --config $k --steps 8 --no-cpu-baseline > gpurun_out/${T}_c$k.json 2> gpurun_out/${T}_c$k.err || { echo BENCH_FAIL $k; tail -20 gpurun_out/${T}_c$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c$k.json').read().strip().splitlines()[-1]); r=d['roofline']
print('c$k', round(d['value']/1e6, 3), 'M/s p50', round(d['p50_ms'], 2), r.get('kernel'), round(r['avg_launch_ms']*1e3, 2), 'us frac', round(r['frac'], 3))"
done
NKM_PROFILE=1 timeout -k 10 400 python bench.py --config 5 --override --steps 4 --warmup 1 > gpurun_out/${T}_c5o.json 2> gpurun_out/${T}_c5o.err || { echo BENCH_FAIL c5o; tail -20 gpurun_out/${T}_c5o.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c5o.json').read().strip().splitlines()[-1])
print('c5o', round(d['value']/1e6, 3), 'M/s p50', round(d['p50_ms'], 2), d['config'].get('override_step_ms'))"
