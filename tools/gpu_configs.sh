# One-GPU bench lines of the other BASELINE configs (parity cases, not the
# headline): C2 100k, C4 500k (one GPU's share of 4M/8), C5 1M RevPrecision,
# C7 100k multi-term.  Lines appended to gpurun_out/configs.jsonl.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/configs.jsonl
for a in "--config 7 --tickets 10000" "--config 5 --tickets 100000"; do
  timeout -k 10 300 python bench.py $a --steps 3 --warmup 1 --no-cpu-baseline >> gpurun_out/configs.jsonl 2> gpurun_out/configs.err || exit 1
done
echo EXIT $?
