# Host-side scaling of the pool replay on the GPU box (no GPU use):
# generic (replay_pool) vs dense (DenseReplay) at 1/8/16 threads.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
{
for d in "" 1; do
echo "== RB_DENSE=$d"
RB_DENSE=$d tools/replay_bench 1000000 5
RB_DENSE=$d tools/replay_bench 1000000 3 8
RB_DENSE=$d RB_POOLS=16 tools/replay_bench 1000000 3 16
RB_DENSE=$d RB_POOLS=16 tools/replay_bench 1000000 3 8
done
} > gpurun_out/cpu_scaling.txt 2>&1
echo EXIT $?
