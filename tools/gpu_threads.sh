set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
(lscpu; echo; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), sorted(os.sched_getaffinity(0)))"; cat /proc/meminfo | head -3) > gpurun_out/cpuinfo.txt 2>&1
for t in 1 4 8 16; do
  NKM_THREADS=$t NKM_PROFILE=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_t$t.json 2> gpurun_out/bench_t$t.err || exit 1
done
echo EXIT $?
