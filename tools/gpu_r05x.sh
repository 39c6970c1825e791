# Round 5: the delivery tests on the GPU (HIP handles, C3 at 1M).  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05x}
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_delivery.py > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAILED|Error|assert" gpurun_out/${T}_tests.log | head -30; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/${T}_tests.log | tail -14
