# Round 5: the headline (C3) and C4 / C5 with this session's library against
# the round's earlier commit 754d06f (ab/libnakama_mm_head.so through
# NKM_LIBRARY), interleaved on one box.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05ao}
line() {
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), 'ms_per_step', round(d['ms_per_step'], 2))" $1 "$2"
}
HEAD_SO=$GRAFT_REPO_ROOT/ab/libnakama_mm_head.so
for cfg in 3 5 4; do
  for k in a b c; do
    [ $cfg = 4 ] && [ $k = c ] && continue
    for v in new old; do
      if [ $v = old ]; then L=$HEAD_SO; else L=; fi
      NKM_LIBRARY=$L NKM_PROFILE=1 timeout -k 10 300 python bench.py --config $cfg --steps 10 --no-cpu-baseline > gpurun_out/${T}_c${cfg}_$v$k.json 2> gpurun_out/${T}_c${cfg}_$v$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c${cfg}_$v$k.err; exit 1; }
      line gpurun_out/${T}_c${cfg}_$v$k.json "c$cfg $v $k"
    done
  done
done
