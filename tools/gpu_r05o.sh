# Round 5: the C3 walk on the box's host alone (tools/replay_bench, no GPU):
# one pool's identity walk warm on one thread, then 8 pools on 16 threads with
# the gather across the threads vs each walk gathering its own pool.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05o}
{
RB_MODE=c3 timeout -k 10 120 tools/replay_bench 1000000 10 0
for k in a b; do
  RB_MODE=c3 RB_IDENT=1 timeout -k 10 120 tools/replay_bench 1000000 5 16
  RB_MODE=c3 RB_IDENT=1 RB_SELFGATHER=1 timeout -k 10 120 tools/replay_bench 1000000 5 16
done
RB_MODE=c3 timeout -k 10 120 tools/replay_bench 1000000 5 16
} > gpurun_out/${T}_replay_bench.txt 2>&1
cat gpurun_out/${T}_replay_bench.txt
