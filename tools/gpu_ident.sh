# Identity pools without the pipelined gather (C4): parity tests, then C4 and C3 phase lines.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-id}
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu -k "full_size or c4 or c3 or pipelined or exact_walk or parallel or multi" --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for C in "--config 4 --steps 4 --warmup 1" "--steps 11 --warmup 2" "--config 4 --steps 4 --warmup 1"; do
  N=c$(echo "$C" | sed 's/--config //;s/ .*//'); [ "$N" = "c--steps" ] && N=c3
  NKM_PROFILE=2 timeout -k 10 300 python bench.py $C --no-cpu-baseline > gpurun_out/${T}_$N.json 2> gpurun_out/${T}_$N.err || { echo "FAIL $N"; tail -20 gpurun_out/${T}_$N.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${T}_$N.json'));r=d['roofline'];print('$N',round(d['value']/1e6,2),round(d['p50_ms'],3),r['kernel'],round(r['frac'],3))"
  grep "pool walks" gpurun_out/${T}_$N.err | tail -1; grep "^\[nkm\] sync" gpurun_out/${T}_$N.err | tail -1 | grep -o "pass [0-9.]* ms\|replay [0-9.]* ms\|finish [0-9.]* ms\|task max [0-9.]* ms\|gather [0-9.]*\|job [0-9.]*\|clear [0-9.]*" | tr '\n' ' '; echo
done
