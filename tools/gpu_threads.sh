# Host-thread sweep of the C3 pass with the phase breakdown (NKM_PROFILE).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
(lscpu; nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; taskset -p $$) > gpurun_out/host_cpu.txt 2>&1 || true
for t in ${NKM_SWEEP:-1 8 16}; do
  NKM_THREADS=$t NKM_PROFILE=1 timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench_t$t.json 2> gpurun_out/bench_t$t.err || exit 1
done
echo EXIT $?
