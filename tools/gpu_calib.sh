# FETCH_SIZE/WRITE_SIZE calibration (tools/fetch_calib) + a phase breakdown of the C3 pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib_fetch -o calib --output-format csv -- tools/fetch_calib > gpurun_out/calib_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/calib_write -o calib --output-format csv -- tools/fetch_calib > gpurun_out/calib_write.log 2>&1 && \
NKM_PROFILE=1 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_phase.json 2> gpurun_out/bench_phase.err
echo EXIT $?
