# Round 5: multi-rank / multi-handle rehearsal on the one-GPU box — 2 ranks
# over gloo sharing device 0 (C3 weak, C5 strong), and one process driving 2
# sub-handles on device 0 (--multi-handle 2, C3 and C4).  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05z}
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533"
for C in 3 5; do
  NKM_BENCH_BACKEND=gloo timeout -k 10 400 $R bench.py --gpus 2 --config $C --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_dist2_c$C.json 2> gpurun_out/${T}_dist2_c$C.err || { echo DIST_FAIL $C; tail -20 gpurun_out/${T}_dist2_c$C.err; exit 1; }
done
for C in 3 4; do
  timeout -k 10 400 python bench.py --multi-handle 2 --config $C --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_mh2_c$C.json 2> gpurun_out/${T}_mh2_c$C.err || { echo MH_FAIL $C; tail -20 gpurun_out/${T}_mh2_c$C.err; exit 1; }
done
for f in dist2_c3 dist2_c5 mh2_c3 mh2_c4; do
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_$f.json').read().strip().splitlines()[-1])
print('$f', d['n_gpus'], round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), d['config'].get('parallelism'), d['config'].get('cluster_phases_ms_rank0'))"
done
