# Quick kernel iteration: the headline bench (3 steps) under rocprofv3's
# kernel-trace summary, once per env setting given in $KB (default: one run
# with the defaults); output under gpurun_out/kb/<n>/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
n=0
for v in ${KB:-NKM_NONE=1}; do
  mkdir -p gpurun_out/kb/$n
  echo "$v" > gpurun_out/kb/$n/env.txt
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kb/$n -o kb --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/kb/$n/bench.json 2> gpurun_out/kb/$n/bench.err || exit $?
  n=$((n+1))
done
echo EXIT 0
