# PMC traffic of one config's dominant eval kernel: one rocprofv3 pass per
# counter (FETCH_SIZE, WRITE_SIZE — they do not fit one pass) over a short
# bench, then tools/pmc_traffic.py -> gpurun_out/<tag>_traffic.json, tagged
# with the config and ticket count bench.py matches it on.
# Usage: tools/gpu_pmc_cfg.sh <tag> <config> <kernel> [tickets]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=$1; C=$2; K=$3
N=${4:-$(python3 -c "import bench; print(bench.DEFAULT_TICKETS.get($C, 1000000))")}
B="python3 bench.py --config $C --tickets $N --steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${T}_fetch -o fetch --output-format csv -- $B > gpurun_out/${T}_fetch.json 2> gpurun_out/${T}_fetch.err || { echo FETCH_FAIL; tail -5 gpurun_out/${T}_fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${T}_write -o write --output-format csv -- $B > gpurun_out/${T}_write.json 2> gpurun_out/${T}_write.err || { echo WRITE_FAIL; tail -5 gpurun_out/${T}_write.err; exit 1; }
python3 tools/pmc_traffic.py --fetch gpurun_out/${T}_fetch --write gpurun_out/${T}_write --kernel "$K" --config $C --tickets $N --out gpurun_out/${T}_traffic.json
