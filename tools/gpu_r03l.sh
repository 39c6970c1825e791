# Every -m gpu test, smoke, the C3 headline (hashed contiguous scan by
# default), C4 and C5 with phase timings, kernel-trace stats of C3.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r03l}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
for C in "" "--config 4 --steps 4 --warmup 1" "--config 5 --steps 6 --warmup 1"; do
  N=c$(echo "$C" | sed 's/--config //;s/ .*//'); [ "$N" = "c" ] && N=c3 && C="--steps 11 --warmup 2"
  NKM_PROFILE=1 timeout -k 10 300 python bench.py $C --no-cpu-baseline > gpurun_out/${T}_$N.json 2> gpurun_out/${T}_$N.err || { echo "FAIL $N"; tail -20 gpurun_out/${T}_$N.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${T}_$N.json'));r=d['roofline'];print('$N',round(d['value']/1e6,1),round(d['p50_ms'],3),r['kernel'],round(r['avg_launch_ms']*1e3,2),round(r['frac'],3))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof3 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_prof3.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/${T}_prof3.log; exit 1; }
head -8 gpurun_out/${T}_prof3/run_kernel_stats.csv
