# Bench lines of one config under several environment settings (NKM_* knobs),
# with the pass phase profile.  $1 = bench arguments, then one argument per
# setting ("" = defaults), e.g.
#   bash tools/gpu_envsweep.sh "--config 2 --tickets 100000" "NKM_WIN=0" ""
# Lines appended to gpurun_out/envsweep.jsonl (each tagged with its setting).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/envsweep.jsonl
: > gpurun_out/envsweep.err
ARGS=$1
shift
for e in "$@"; do
  echo "== $e" >> gpurun_out/envsweep.err
  env $e NKM_PROFILE=1 timeout -k 10 300 python bench.py $ARGS --steps 3 --warmup 1 --no-cpu-baseline 2>> gpurun_out/envsweep.err | sed "s/^{/{\"env\": \"$e\", /" >> gpurun_out/envsweep.jsonl || exit 1
done
echo EXIT $?
