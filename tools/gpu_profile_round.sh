# Round profile set for the headline bench (C3 1M): rocprofv3 kernel-trace
# stats, then one PMC pass per counter group (FETCH_SIZE, WRITE_SIZE, SQ/GRBM)
# of the same command, then the other configs' bench lines.  $1 = round tag
# (output under gpurun_out/prof_$1_*).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02}
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_trace -o trace --output-format csv -- $B > gpurun_out/prof_${T}_trace.json 2> gpurun_out/prof_${T}_trace.err && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_${T}_fetch -o fetch --output-format csv -- $B > gpurun_out/prof_${T}_fetch.json 2> gpurun_out/prof_${T}_fetch.err && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_${T}_write -o write --output-format csv -- $B > gpurun_out/prof_${T}_write.json 2> gpurun_out/prof_${T}_write.err && \
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/prof_${T}_sq -o sq --output-format csv -- $B > gpurun_out/prof_${T}_sq.json 2> gpurun_out/prof_${T}_sq.err
rc=$?
echo "profile EXIT $rc"
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_configs.sh "$2"
