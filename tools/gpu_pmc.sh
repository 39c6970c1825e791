# GPU tests, kernel-trace stats of the bench, and PMC passes (one counter
# group per run: FETCH_SIZE, WRITE_SIZE, SQ/GRBM utilisation) for the
# dominant query-eval kernel.  Output under gpurun_out/pmc_*.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_trace -o trace --output-format csv -- $B > gpurun_out/pmc_trace.json 2> gpurun_out/pmc_trace.err && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o fetch --output-format csv -- $B > gpurun_out/pmc_fetch.json 2> gpurun_out/pmc_fetch.err && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o write --output-format csv -- $B > gpurun_out/pmc_write.json 2> gpurun_out/pmc_write.err && \
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq -o sq --output-format csv -- $B > gpurun_out/pmc_sq.json 2> gpurun_out/pmc_sq.err
echo EXIT $?
