# Quick kernel iteration: the headline bench (3 steps) under rocprofv3's
# kernel-trace summary; output under gpurun_out/kb/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/kb
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kb -o kb --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/kb/bench.json 2> gpurun_out/kb/bench.err
echo EXIT $?
