# Same-tree A/B of environment settings on one box: for each ';'-separated
# bench argument set in $1, runs every env setting of $ENVS (space-separated,
# NAME=value, "-" = none), alternating, $ROUNDS times.  Lines tagged with the
# env and the arguments in gpurun_out/envab.jsonl, phases in envab.err.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/envab.jsonl
: > gpurun_out/envab.err
IFS=';' read -ra SETS <<< "$1"
for a in "${SETS[@]}"; do
  for i in $(seq 1 ${ROUNDS:-2}); do
    for v in $ENVS; do
      e=$v; [ "$v" = "-" ] && e="NKM_NONE=1"
      echo "== $v $a" >> gpurun_out/envab.err
      env $e NKM_PROFILE=1 timeout -k 10 300 python bench.py $a --steps 8 --warmup 2 --no-cpu-baseline 2>> gpurun_out/envab.err | sed "s/^{/{\"tree\": \"$v\", \"args\": \"$a\", /" >> gpurun_out/envab.jsonl || exit 1
    done
  done
done
echo EXIT $?
