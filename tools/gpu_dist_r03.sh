# Rehearsal of bench.py's multi-rank path on a one-GPU box (2 ranks over
# gloo sharing device 0; the driver's 8-GPU runs use RCCL, one GPU per rank):
# C3 weak and C5 strong, with each step's cluster phases (local pass,
# summary, merge) on rank 0, and the 1-rank C3 line.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-dist}
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533"
NKM_BENCH_BACKEND=gloo timeout -k 10 500 $R bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.err || { echo C3_FAIL; tail -20 gpurun_out/${T}_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_c3.json'));print('C3x2',round(d['value']/1e6,1),round(d['p50_ms'],2),d['config'].get('cluster_phases_ms_rank0'))"
NKM_BENCH_BACKEND=gloo timeout -k 10 500 $R bench.py --gpus 2 --steps 4 --warmup 1 --config 5 --no-cpu-baseline > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.err || { echo C5_FAIL; tail -20 gpurun_out/${T}_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_c5.json'));print('C5x2',round(d['value']/1e6,1),round(d['p50_ms'],2),d['config'].get('cluster_phases_ms_rank0'))"
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c3x1.json 2> gpurun_out/${T}_c3x1.err || { echo C3X1_FAIL; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_c3x1.json'));print('C3x1',round(d['value']/1e6,1),round(d['p50_ms'],2))"
