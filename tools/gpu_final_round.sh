# End-of-round measurement set of the current tree ($1 = tag, default r02c):
# -m gpu tests, smoke, the headline bench (with the CPU baseline), rocprofv3
# kernel-trace stats of the bench, FETCH_SIZE / WRITE_SIZE passes of it (one
# counter per run) -> mscan traffic JSON, the other configs' bench lines, and
# PMC traffic of search_kernel<512> (C2) and rsmall_kernel (C5).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02c}
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
NKM_PROFILE=1 timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trace -o trace --output-format csv -- $B > gpurun_out/${T}_trace.json 2> gpurun_out/${T}_trace.err || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${T}_fetch -o fetch --output-format csv -- $B > gpurun_out/${T}_fetch.json 2> gpurun_out/${T}_fetch.err || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${T}_write -o write --output-format csv -- $B > gpurun_out/${T}_write.json 2> gpurun_out/${T}_write.err || exit $?
python3 tools/pmc_traffic.py --fetch gpurun_out/${T}_fetch --write gpurun_out/${T}_write --kernel mscan_kernel --out gpurun_out/${T}_traffic.json > /dev/null || exit $?
bash tools/gpu_configs.sh "--config 1 --tickets 10000;--config 2 --tickets 100000;--config 4;--config 5;--config 5 --override;--config 7 --tickets 10000" || exit $?
bash tools/gpu_pmc_configs.sh
echo "FINAL EXIT $?"
