# GPU parity tests, then the variable-score-heavy bench lines (C7 multi-term
# 10k, C2 skill windows 100k) and the C3 headline for regressions.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
: > gpurun_out/vark.jsonl
for a in "--config 7 --tickets 10000" "--config 2 --tickets 100000" "--config 1 --tickets 10000" "--config 3"; do
  NKM_PROFILE=1 timeout -k 10 300 python bench.py $a --steps 3 --warmup 1 --no-cpu-baseline >> gpurun_out/vark.jsonl 2>> gpurun_out/vark.err || exit 1
done
echo EXIT $?
