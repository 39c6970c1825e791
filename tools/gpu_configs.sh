# One-GPU bench lines of the other BASELINE configs (parity cases, not the
# headline), with the pass phase profile (NKM_PROFILE) on stderr:
# C2 100k, C4 4M (its whole set on one GPU), C5 1M RevPrecision, C7 10k
# multi-term.  Lines appended to gpurun_out/configs.jsonl; $1 overrides the list
# (';'-separated argument sets).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/configs.jsonl
: > gpurun_out/configs.err
LIST=${1:-"--config 2 --tickets 100000;--config 4;--config 5;--config 7 --tickets 10000"}
IFS=';' read -ra SETS <<< "$LIST"
for a in "${SETS[@]}"; do
  echo "== $a" >> gpurun_out/configs.err
  NKM_PROFILE=1 timeout -k 10 400 python bench.py $a --steps 3 --warmup 1 --no-cpu-baseline >> gpurun_out/configs.jsonl 2>> gpurun_out/configs.err || exit 1
done
echo EXIT $?
