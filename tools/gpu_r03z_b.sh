# End-of-round set, part B: the driver's default bench line (with the CPU
# baseline), C3 / C4 / C5 / C2 with phase timings, kernel-trace stats of C3,
# PMC traffic of C3's eval kernel.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r03z}
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_bench.json'));r=d['roofline'];c=d['cpu_baseline'];print('bench',round(d['value']/1e6,1),round(d['ms_per_step'],3),r['kernel'],round(r['frac'],3),c['value'],c['kind'])"
for C in "--steps 11 --warmup 2" "--config 4 --steps 4 --warmup 1" "--config 5 --steps 6 --warmup 1" "--config 2 --steps 4 --warmup 1"; do
  N=c$(echo "$C" | sed 's/--config //;s/ .*//'); [ "$N" = "c--steps" ] && N=c3
  NKM_PROFILE=1 timeout -k 10 300 python bench.py $C --no-cpu-baseline > gpurun_out/${T}_$N.json 2> gpurun_out/${T}_$N.err || { echo "FAIL $N"; tail -20 gpurun_out/${T}_$N.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${T}_$N.json'));r=d['roofline'];print('$N',round(d['value']/1e6,2),round(d['p50_ms'],3),r['kernel'],round(r['avg_launch_ms']*1e3,2),round(r['frac'],3))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof3 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_prof3.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/${T}_prof3.log; exit 1; }
head -6 gpurun_out/${T}_prof3/run_kernel_stats.csv
bash tools/gpu_pmc_c3.sh ${T}_pmc && cat gpurun_out/${T}_pmc_traffic.json
