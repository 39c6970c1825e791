# Kernel-trace stats and PMC traffic passes (FETCH_SIZE, WRITE_SIZE: one
# counter per run) of the variable-score / RevPrecision configs' bench
# commands: C2 100k (search_kernel<512>) and C5 1M (rsmall_kernel).
# Output under gpurun_out/pmcc_<tag>_*; traffic JSON via tools/pmc_traffic.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # $1 tag, $2 kernel name, rest: bench args
  local T=$1 K=$2; shift 2
  local B="python3 bench.py $* --steps 2 --warmup 1 --no-cpu-baseline"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pmcc_${T}_trace -o trace --output-format csv -- $B > gpurun_out/pmcc_${T}_trace.json 2> gpurun_out/pmcc_${T}_trace.err && \
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcc_${T}_fetch -o fetch --output-format csv -- $B > gpurun_out/pmcc_${T}_fetch.json 2> gpurun_out/pmcc_${T}_fetch.err && \
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcc_${T}_write -o write --output-format csv -- $B > gpurun_out/pmcc_${T}_write.json 2> gpurun_out/pmcc_${T}_write.err && \
  python3 tools/pmc_traffic.py --fetch gpurun_out/pmcc_${T}_fetch --write gpurun_out/pmcc_${T}_write --kernel $K --out gpurun_out/pmcc_${T}_traffic.json > /dev/null
}
run c2 "search_kernel<512>" --config 2 --tickets 100000 && \
run c5 rsmall_kernel --config 5
echo EXIT $?
