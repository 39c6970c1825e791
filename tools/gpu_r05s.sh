# Round 5: C3 merge cost — the pipelined merge (default) vs the merge after all
# walks (NKM_PIPE=0, its time alone on 16 workers), interleaved.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05s}
for k in 1a 0a 1b 0b; do
  P=${k:0:1}
  NKM_PIPE=$P NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 3 --steps 10 --no-cpu-baseline > gpurun_out/${T}_c3_$k.json 2> gpurun_out/${T}_c3_$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c3_$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c3_$k.json').read().strip().splitlines()[-1])
print('pipe $k', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), 'ms_per_step', round(d['ms_per_step'], 2))"
  grep -E "pass [0-9.]+ ms" gpurun_out/${T}_c3_$k.err | tail -2 | sed 's/.*par bucket/par bucket/; s/| batch.*replay:/| replay:/'
  grep -E "pool walks" gpurun_out/${T}_c3_$k.err | tail -2 | sed 's/.*sum: //; s/gather+reset.*last/last/'
done
