# Finish-phase timings: C5 and C3 benches at NKM_PROFILE=2.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-f}
NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 5 --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.err || { echo C5_FAIL; tail -20 gpurun_out/${T}_c5.err; exit 1; }
NKM_PROFILE=2 timeout -k 10 300 python bench.py --steps 11 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.err || { echo C3_FAIL; tail -20 gpurun_out/${T}_c3.err; exit 1; }
grep -h "finish:" gpurun_out/${T}_c5.err gpurun_out/${T}_c3.err | tail -8
for c in c5 c3; do python -c "import json;d=json.load(open('gpurun_out/${T}_$c.json'));print('$c',d['value']/1e6,d['p50_ms'])"; done
