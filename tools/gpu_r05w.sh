# Round 5: rocprofv3 kernel-trace summaries of the C3 / C5 / C2 lines and the
# C5 rpack PMC traffic (u8 entry positions), then the C4, C5, C2 and C5 +
# override lines.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05w}
for C in 3 5 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c${C}_prof -o run -- python3 bench.py --config $C --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c${C}_prof.log 2>&1 || { echo PROF_FAIL $C; tail -20 gpurun_out/${T}_c${C}_prof.log; exit 1; }
  head -5 gpurun_out/${T}_c${C}_prof/run_kernel_stats.csv | cut -c1-160
done
bash tools/gpu_pmc_cfg.sh ${T}_c5 5 rpack_kernel || exit 1
cat gpurun_out/${T}_c5_traffic.json; echo
for k in 4 5 2; do
  NKM_PROFILE=1 timeout -k 10 400 python bench.py --config $k --steps 8 --no-cpu-baseline --traffic gpurun_out/${T}_c5_traffic.json > gpurun_out/${T}_c$k.json 2> gpurun_out/${T}_c$k.err || { echo BENCH_FAIL $k; tail -20 gpurun_out/${T}_c$k.err; exit 1; }
done
NKM_PROFILE=1 timeout -k 10 400 python bench.py --config 5 --override --steps 4 --warmup 1 > gpurun_out/${T}_c5o.json 2> gpurun_out/${T}_c5o.err || { echo BENCH_FAIL c5o; tail -20 gpurun_out/${T}_c5o.err; exit 1; }
for f in c4 c5 c2 c5o; do
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_$f.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', round(d['value']/1e6, 3), 'M/s p50', round(d['p50_ms'], 2), r.get('kernel'), round(r['avg_launch_ms']*1e3, 2), 'us frac', round(r['frac'], 3), 'traffic', r.get('traffic'), d['config'].get('override_step_ms'), (d.get('cpu_baseline') or {}).get('value'))"
done
