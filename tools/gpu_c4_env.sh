# C4 phase lines under host-path switches (default, 8 threads, no pipelined merge, generic walk).  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-c4e}
for v in "X=0" "NKM_THREADS=8" "NKM_PIPE=0" "NKM_DENSE=0" "X=0"; do
env $v NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c4.json 2> gpurun_out/${T}_c4_$v.err || { echo C4_FAIL; tail -20 gpurun_out/${T}_c4_$v.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_c4.json'));print('C4 $v',round(d['value']/1e6,1),round(d['p50_ms'],2))"
grep "pool walks" gpurun_out/${T}_c4_$v.err | tail -1; grep "^\[nkm\] sync" gpurun_out/${T}_c4_$v.err | tail -1 | grep -o "pass [0-9.]* ms\|replay [0-9.]* ms\|finish [0-9.]* ms\|task max [0-9.]* ms\|merge [0-9.]* ms\|gather [0-9.]*\|job [0-9.]*" | tr '\n' ' '; echo
done
