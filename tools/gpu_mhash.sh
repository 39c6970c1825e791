# GPU call for the hashed mscan: its parity tests (C4 64 signatures, C3/C1
# forced), C4 and C3 benches with per-phase timings, and a kernel-trace
# profile of the C4 bench.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-mh}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "hashed or c3_c4 or many_pools or c3_parties" --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for V in "NKM_MCONTIG=1" "NKM_MCONTIG=1 NKM_MCONTIG_J=4" "NKM_MCONTIG=0"; do
  env $V NKM_PROFILE=1 timeout -k 10 300 python bench.py --config 4 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c4.json 2> gpurun_out/${T}_c4.err || { echo BENCH4_FAIL; tail -20 gpurun_out/${T}_c4.err; exit 1; }
  echo "C4 $V"; python -c "import json;d=json.load(open('gpurun_out/${T}_c4.json'));r=d['roofline'];print(d['p50_ms'],r['kernel'],r['avg_launch_ms'],r['frac'])"
  env $V NKM_MHASH=1 timeout -k 10 300 python bench.py --steps 11 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_c3h.json 2> gpurun_out/${T}_c3h.err || { echo BENCH3_FAIL; tail -20 gpurun_out/${T}_c3h.err; exit 1; }
  echo "C3 hashed $V"; python -c "import json;d=json.load(open('gpurun_out/${T}_c3h.json'));r=d['roofline'];print(d['p50_ms'],r['kernel'],r['avg_launch_ms'],r['frac'])"
done
timeout -k 10 300 python bench.py --steps 11 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.err || { echo BENCH3_FAIL; exit 1; }
echo "C3 default"; python -c "import json;d=json.load(open('gpurun_out/${T}_c3.json'));r=d['roofline'];print(d['p50_ms'],r['kernel'],r['avg_launch_ms'],r['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof4 -o run -- python3 bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_prof4.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/${T}_prof4.log; exit 1; }
find gpurun_out/${T}_prof4 -name "*kernel_stats.csv" | head -1 | xargs head -14
