# Same-box A/B of two builds of libnakama_mm.so (tools/ab/libA.so, libB.so):
# alternates them under one bench command.  $1 = tag, $2 = config, $3 = rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1; C=$2; R=${3:-2}
cp nakama_amd/libnakama_mm.so gpurun_out/.lib_keep.so
for r in $(seq 1 $R); do
  for v in A B; do
    cp tools/ab/lib$v.so nakama_amd/libnakama_mm.so
    NKM_PROFILE=1 timeout -k 10 300 python bench.py --config $C --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_${v}$r.json 2> gpurun_out/${T}_${v}$r.err || { echo BENCH_FAIL $v $r; cp gpurun_out/.lib_keep.so nakama_amd/libnakama_mm.so; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_${v}$r.json').read().strip().splitlines()[-1]); print('$v$r', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), 'ms/step', round(d['ms_per_step'], 2))"
  done
done
cp gpurun_out/.lib_keep.so nakama_amd/libnakama_mm.so
rm -f gpurun_out/.lib_keep.so
