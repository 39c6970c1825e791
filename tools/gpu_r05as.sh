# Round 5: C2 100k phase profile (range batch split) x2.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05as}
for k in a b; do
  NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 2 --steps 10 --no-cpu-baseline > gpurun_out/${T}_c2_$k.json 2> gpurun_out/${T}_c2_$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c2_$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c2_$k.json').read().strip().splitlines()[-1])
print('c2 $k', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2))"
  grep -E "\(range\)|pass [0-9.]+ ms" gpurun_out/${T}_c2_$k.err | tail -4 | cut -c1-600
done
