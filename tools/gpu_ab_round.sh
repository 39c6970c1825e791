# Same-box A/B of the headline bench: other trees (git worktrees, default the
# round-start tree ab_old/) against this tree, alternating, with the pass
# phase profile on stderr.  $AB_TREES overrides the list (space-separated,
# "." = this tree); $AB_ROUNDS the number of alternations (default 2).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab.jsonl
: > gpurun_out/ab.err
for i in $(seq 1 ${AB_ROUNDS:-2}); do
  for t in ${AB_TREES:-ab_old .}; do
    echo "== $t" >> gpurun_out/ab.err
    (cd $t && NKM_PROFILE=1 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline | sed "s/^{/{\"tree\": \"$t\", /") >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err || exit 1
  done
done
echo EXIT $?
