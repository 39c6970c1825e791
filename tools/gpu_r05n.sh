# Round 5: hashed-scan chunk shape A/B in the product (NKM_MCONTIG_J=4 vs 8)
# on C3 and C4, interleaved; kernel time from the bench's event pair.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05n}
for k in 3_4a 3_8a 4_4a 4_8a 3_4b 3_8b 4_4b 4_8b; do
  C=${k:0:1}; J=${k:2:1}
  NKM_MCONTIG_J=$J timeout -k 10 300 python bench.py --config $C --steps 10 --no-cpu-baseline > gpurun_out/${T}_c$k.json 2> gpurun_out/${T}_c$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c$k.json').read().strip().splitlines()[-1]); r=d['roofline']
print('c$k', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), r.get('kernel'), round(r['avg_launch_ms']*1e3, 2), 'us frac', round(r['frac'], 3))"
done
