# Rehearses bench.py's multi-rank path on a one-GPU box: 2 ranks over gloo
# sharing device 0 (the driver's 8-GPU runs use RCCL, one GPU per rank).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
NKM_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/dist2.json 2> gpurun_out/dist2.err && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/dist1.json 2> gpurun_out/dist1.err
echo EXIT $?
