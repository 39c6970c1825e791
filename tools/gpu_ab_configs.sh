# Same-box A/B of several bench configs: ab_old/ (a baseline worktree) vs this
# tree, alternating per config; lines tagged with the tree and the arguments.
# $1 overrides the ';'-separated argument sets.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/abc.jsonl
: > gpurun_out/abc.err
LIST=${1:-"--config 2 --tickets 100000;--config 4;--config 5;--config 3"}
IFS=';' read -ra SETS <<< "$LIST"
for a in "${SETS[@]}"; do
  for t in ${AB_TREES:-ab_old . ab_old .}; do
    echo "== $t $a" >> gpurun_out/abc.err
    (cd $t && NKM_PROFILE=1 timeout -k 10 300 python bench.py $a --steps ${ABSTEPS:-8} --warmup 2 --no-cpu-baseline | sed "s/^{/{\"tree\": \"$t\", \"args\": \"$a\", /") >> gpurun_out/abc.jsonl 2>> gpurun_out/abc.err || exit 1
  done
done
echo EXIT $?
