# PMC traffic of the C3 headline's eval kernel: one rocprofv3 pass per
# counter (FETCH_SIZE, WRITE_SIZE) over a short bench, then
# tools/pmc_traffic.py -> gpurun_out/$1_traffic.json (bench.py --traffic).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-pmc3}
K=${2:-mscan_hash_kernel}
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${T}_fetch -o fetch --output-format csv -- $B > gpurun_out/${T}_fetch.json 2> gpurun_out/${T}_fetch.err || { echo FETCH_FAIL; tail -5 gpurun_out/${T}_fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${T}_write -o write --output-format csv -- $B > gpurun_out/${T}_write.json 2> gpurun_out/${T}_write.err || { echo WRITE_FAIL; tail -5 gpurun_out/${T}_write.err; exit 1; }
python3 tools/pmc_traffic.py --fetch gpurun_out/${T}_fetch --write gpurun_out/${T}_write --kernel "$K" --out gpurun_out/${T}_traffic.json
