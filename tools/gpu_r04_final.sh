# Round-4 end-of-round set, part A: the GPU test suite, smoke(), the
# default bench line (C3, with its CPU baseline) and the other configs' lines
# (C2 / C4 / C5 with CPU baselines, C5 + override, C3 and C4 through one
# multi-device handle).  $1 = tag.  Every step under its own time limit; the
# first failure ends the script.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r04z}
timeout -k 10 900 python -u -m pytest -q --timeout 400 --timeout-method thread tests -m gpu > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
NKM_PROFILE=1 timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_bench.err; exit 1; }
for C in 2 4 5; do
  NKM_PROFILE=1 timeout -k 10 400 python bench.py --config $C --steps 8 --warmup 2 > gpurun_out/${T}_c$C.json 2> gpurun_out/${T}_c$C.err || { echo BENCH_FAIL $C; tail -20 gpurun_out/${T}_c$C.err; exit 1; }
done
timeout -k 10 300 python bench.py --config 5 --override --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c5o.json 2> gpurun_out/${T}_c5o.err || { echo BENCH_FAIL c5o; exit 1; }
for C in 3 4; do
  timeout -k 10 300 python bench.py --config $C --multi-handle 2 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_mh2_c$C.json 2> gpurun_out/${T}_mh2_c$C.err || { echo BENCH_FAIL mh2 $C; tail -20 gpurun_out/${T}_mh2_c$C.err; exit 1; }
done
for f in bench c2 c4 c5 c5o mh2_c3 mh2_c4; do
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_$f.json').read().strip().splitlines()[-1]); r=d['roofline']; cb=d.get('cpu_baseline') or {}
print('$f', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), r.get('kernel'), 'frac', round(r['frac'], 3), 'cpu', cb.get('value'))"
done
