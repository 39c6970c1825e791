set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || exit 1
for cfg in "16 0" "1 0" "16 1"; do
  set -- $cfg
  NKM_THREADS=$1 NKM_PIN=$2 NKM_PROFILE=1 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_t$1_p$2.json 2> gpurun_out/bench_t$1_p$2.err || exit 1
done
echo EXIT $?
