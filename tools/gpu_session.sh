# One GPU call: the mscan roof microbenchmark, the -m gpu parity tests (an
# assertion failure, exit 1, does not stop the call; a fault, abort or time
# limit does), smoke, then same-box A/B of the configs (ab_old/ vs this tree).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/mscan_roof > gpurun_out/mscan_roof.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
[ "${AB:-1}" = "1" ] && bash tools/gpu_ab_configs.sh "$ABLIST"
echo "TESTS rc=$rc"
