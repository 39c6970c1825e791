# One GPU call: the -m gpu parity tests (optionally a subset: $1 = -k expr),
# then smoke and a short headline bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
K=${1:+-k "$1"}
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread $K > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
NKM_PROFILE=1 timeout -k 10 600 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
tail -3 gpurun_out/gpu_tests.log
echo EXIT $rc
