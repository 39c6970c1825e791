# Rehearses the multi-GPU front on a one-GPU box: the gpu-marked cluster and
# concurrency tests, then bench.py over 2 ranks (gloo, sharing device 0; the
# driver's 8-GPU runs use RCCL, one GPU per rank) for C3 (weak), C4 and C5
# (strong), C5 with the override hand-off per rank, and the 1-rank C3 line
# for comparison.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533"
timeout -k 10 600 python -u -m pytest tests/test_cluster.py tests/test_concurrency.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/cluster_tests.log 2>&1 && \
NKM_BENCH_BACKEND=gloo timeout -k 10 500 $R bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/dist2_c3.json 2> gpurun_out/dist2_c3.err && \
NKM_BENCH_BACKEND=gloo timeout -k 10 500 $R bench.py --gpus 2 --steps 3 --warmup 1 --config 4 --tickets 1000000 > gpurun_out/dist2_c4.json 2> gpurun_out/dist2_c4.err && \
NKM_BENCH_BACKEND=gloo timeout -k 10 500 $R bench.py --gpus 2 --steps 3 --warmup 1 --config 5 > gpurun_out/dist2_c5.json 2> gpurun_out/dist2_c5.err && \
NKM_BENCH_BACKEND=gloo timeout -k 10 500 $R bench.py --gpus 2 --steps 2 --warmup 1 --config 5 --override --no-cpu-baseline > gpurun_out/dist2_c5o.json 2> gpurun_out/dist2_c5o.err && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/dist1.json 2> gpurun_out/dist1.err
rc=$?
tail -2 gpurun_out/cluster_tests.log
echo EXIT $rc
