# Round-3 first GPU call: the new tests first (multi handle, >=63 hits,
# full-size digests), then every -m gpu test, smoke, a short bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_multi.py tests/test_full_size_golden.py tests/test_gpu_parity.py -x -v -m gpu -k "multi or full_size or 63_hits" --timeout 300 --timeout-method thread > gpurun_out/r03a_new_tests.log 2>&1 || { echo NEW_FAIL; tail -30 gpurun_out/r03a_new_tests.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r03a_gpu_tests.log 2>&1 || { echo ALL_FAIL; tail -30 gpurun_out/r03a_gpu_tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03a_smoke.log 2>&1 || exit 1
NKM_PROFILE=1 timeout -k 10 300 python bench.py --steps 7 --warmup 2 --no-cpu-baseline > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err
echo EXIT $?
tail -3 gpurun_out/r03a_gpu_tests.log
