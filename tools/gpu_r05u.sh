# Round 5: C3 job-start latency — the finish retire job's and the assembly
# count sweep's own task times vs their walls (NKM_PROFILE=2), with and
# without the workers' pre-wake.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05u}
for k in 1a 0a 1b 0b; do
  W=${k:0:1}
  NKM_PREWAKE=$W NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 3 --steps 10 --no-cpu-baseline > gpurun_out/${T}_c3_$k.json 2> gpurun_out/${T}_c3_$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c3_$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c3_$k.json').read().strip().splitlines()[-1])
print('prewake $k', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), 'ms_per_step', round(d['ms_per_step'], 2))"
  grep -E "finish: retire|count sweep" gpurun_out/${T}_c3_$k.err | tail -4
done
NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 4 --steps 4 --no-cpu-baseline > gpurun_out/${T}_c4.json 2> gpurun_out/${T}_c4.err || { echo BENCH_FAIL c4; tail -20 gpurun_out/${T}_c4.err; exit 1; }
NKM_PIPE=0 NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 4 --steps 4 --no-cpu-baseline > gpurun_out/${T}_c4_pipe0.json 2> gpurun_out/${T}_c4_pipe0.err || { echo BENCH_FAIL c4; tail -20 gpurun_out/${T}_c4_pipe0.err; exit 1; }
for f in c4 c4_pipe0; do
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_$f.json').read().strip().splitlines()[-1])
print('$f', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2))"
  grep -E "pool walks|pass [0-9.]+ ms" gpurun_out/${T}_$f.err | tail -2 | sed 's/.*sum: //; s/| batch.*replay:/| replay:/' | cut -c1-400
done
