# Round 5: C3 worker placement A/B — node-wide (default) vs one CPU each
# (NKM_PIN=1: physical cores first), interleaved, with the walk / merge split.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05t}
for k in da 1a db 1b dc 1c; do
  P=${k:0:1}
  if [ "$P" = "1" ]; then export NKM_PIN=1; else unset NKM_PIN; fi
  NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 3 --steps 10 --no-cpu-baseline > gpurun_out/${T}_c3_$k.json 2> gpurun_out/${T}_c3_$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c3_$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c3_$k.json').read().strip().splitlines()[-1])
print('pin $k', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), 'ms_per_step', round(d['ms_per_step'], 2))"
  grep -E "pool walks" gpurun_out/${T}_c3_$k.err | tail -3 | sed 's/.*sum: //; s/gather+reset.*last/last/' || true
done
