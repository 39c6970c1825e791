# GPU parity tests + a short bench with phase breakdown + kernel-trace stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
NKM_PROFILE=1 timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profq -o trace --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_qt.json 2> gpurun_out/bench_qt.err
echo EXIT $?
