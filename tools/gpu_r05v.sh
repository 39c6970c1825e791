# Round 5 checkpoint: the whole GPU suite, smoke(), the default bench line
# (C3, with its cpu_baseline), then rocprofv3 kernel-trace summaries of C3
# and C5 and the C5 rpack PMC traffic (u8 entry positions).  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05v}
timeout -k 10 1100 python -u -m pytest -q --timeout 400 --timeout-method thread tests -m gpu > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error" gpurun_out/${T}_gpu_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_bench.err; exit 1; }
tail -1 gpurun_out/${T}_bench.json
