# Round 5: hardware counters around the C3 identity walk on the box's host
# (tools/replay_bench RB_PERF=1; no GPU).  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05p}
{
cat /proc/sys/kernel/perf_event_paranoid
RB_MODE=c3 RB_PERF=1 timeout -k 10 120 tools/replay_bench 1000000 20 0
RB_MODE=c3 RB_PERF=1 timeout -k 10 120 tools/replay_bench 1000000 20 0
RB_MODE=c4 RB_PERF=1 timeout -k 10 120 tools/replay_bench 4000000 10 0
} > gpurun_out/${T}_walk_perf.txt 2>&1
cat gpurun_out/${T}_walk_perf.txt
