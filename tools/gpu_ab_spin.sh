# Same-box A/B of the host workers' spin window (NKM_SPIN_US) on the C3
# headline, the C5 phases after the plan_pools fix, and PMC traffic of
# rpack_kernel (FETCH_SIZE / WRITE_SIZE passes, one counter per run).  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-ab}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "packed or c5 or c3 or c4_many" --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for S in 0 30 200 0 30 200; do
  NKM_SPIN_US=$S NKM_PROFILE=2 timeout -k 10 300 python bench.py --steps 11 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_c3_s$S.json 2> gpurun_out/${T}_c3_s$S.err || { echo C3_FAIL; tail -20 gpurun_out/${T}_c3_s$S.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${T}_c3_s$S.json'));print('C3 spin $S',round(d['value']/1e6,1),round(d['p50_ms'],3))"
done
NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 5 --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.err || { echo C5_FAIL; tail -20 gpurun_out/${T}_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_c5.json'));r=d['roofline'];print('C5',d['value']/1e6,d['p50_ms'],r['kernel'],r['avg_launch_ms'],r['frac'])"
B="python3 bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${T}_fetch -o fetch --output-format csv -- $B > gpurun_out/${T}_fetch.json 2> gpurun_out/${T}_fetch.err || { echo FETCH_FAIL; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${T}_write -o write --output-format csv -- $B > gpurun_out/${T}_write.json 2> gpurun_out/${T}_write.err || { echo WRITE_FAIL; exit 1; }
python3 tools/pmc_traffic.py --fetch gpurun_out/${T}_fetch --write gpurun_out/${T}_write --kernel "rpack_kernel<8>" --out gpurun_out/${T}_rpack_traffic.json && cat gpurun_out/${T}_rpack_traffic.json
