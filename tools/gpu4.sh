set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
NKM_PROFILE=1 timeout -k 10 600 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
echo EXIT $?
