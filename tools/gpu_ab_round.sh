# Same-box A/B of the headline bench: the round-start tree (ab_old/, a git
# worktree of the round-1 commit) against this tree, alternating, with the
# pass phase profile on stderr.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab.jsonl
: > gpurun_out/ab.err
for i in 1 2; do
  for t in ab_old .; do
    echo "== $t" >> gpurun_out/ab.err
    (cd $t && NKM_PROFILE=1 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline | sed "s/^{/{\"tree\": \"$t\", /") >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err || exit 1
  done
done
echo EXIT $?
