# Round-4 measurement set: kernel-trace stats and PMC traffic of each
# config's dominant eval kernel, then bench lines that pick the traffic files
# up.  $1 = tag, $2 = "config:kernel ..." (default C3 and C4's
# mscan_hash_kernel).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r04p}
PAIRS=${2:-"3:mscan_hash_kernel 4:mscan_hash_kernel"}
for P in $PAIRS; do
  C=${P%%:*}; K=${P#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c${C}_prof -o run -- python3 bench.py --config $C --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c${C}_prof.log 2>&1 || { echo PROF_FAIL $C; tail -20 gpurun_out/${T}_c${C}_prof.log; exit 1; }
  head -8 gpurun_out/${T}_c${C}_prof/run_kernel_stats.csv
  bash tools/gpu_pmc_cfg.sh ${T}_c${C} $C $K || exit 1
  cat gpurun_out/${T}_c${C}_traffic.json
  cp gpurun_out/${T}_c${C}_traffic.json profiles/r04_c${C}_traffic.json
  NKM_PROFILE=1 timeout -k 10 300 python bench.py --config $C --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c${C}.json 2> gpurun_out/${T}_c${C}.err || { echo BENCH_FAIL $C; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${T}_c${C}.json'));r=d['roofline'];print('c$C',round(d['value']/1e6,1),round(d['p50_ms'],2),r['kernel'],round(r['avg_launch_ms']*1e3,2),'us',round(r['bytes_per_launch']/1e6,2),'MB frac',round(r['frac'],3),'traffic',r['traffic'])"
done
