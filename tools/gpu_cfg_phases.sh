# Phase timings (NKM_PROFILE=2) of the non-headline configs and a kernel-trace
# profile of C5: where the C5 / C5+override / C2 passes spend their time.
# $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-cfg}
for C in "--config 5" "--config 5 --override" "--config 2 --tickets 100000"; do
  N=$(echo $C | tr -d ' -')
  NKM_PROFILE=2 timeout -k 10 300 python bench.py $C --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_${N}.json 2> gpurun_out/${T}_${N}.err || { echo "FAIL $C"; tail -20 gpurun_out/${T}_${N}.err; exit 1; }
  echo "== $C"; python -c "import json;d=json.load(open('gpurun_out/${T}_${N}.json'));r=d['roofline'];print(d['value'],d['p50_ms'],r['kernel'],r['avg_launch_ms'],r['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof5 -o run -- python3 bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_prof5.log 2>&1 || { echo PROF5_FAIL; tail -20 gpurun_out/${T}_prof5.log; exit 1; }
head -12 gpurun_out/${T}_prof5/run_kernel_stats.csv
