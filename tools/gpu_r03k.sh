# Every -m gpu test on the tree with the RevPrecision fast walk and the
# parallel windowed assembly, then C5 / C2 benches with phases and the C3
# mscan / hashed A/B.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r03k}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 5 --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.err || { echo C5_FAIL; tail -20 gpurun_out/${T}_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_c5.json'));r=d['roofline'];print('C5',d['value']/1e6,d['p50_ms'],r['kernel'],r['avg_launch_ms'],r['frac'])"
NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 2 --tickets 100000 --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c2.json 2> gpurun_out/${T}_c2.err || { echo C2_FAIL; tail -20 gpurun_out/${T}_c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_c2.json'));r=d['roofline'];print('C2',d['value']/1e6,d['p50_ms'],r['kernel'],r['avg_launch_ms'],r['frac'])"
grep "pass" gpurun_out/${T}_c2.err | tail -2 | cut -c1-300
bash tools/gpu_ab_mhash_c3.sh ${T}m
