# GPU call for the C2 host work: the parity tests that cover variable-score
# batches, restarts and the parallel assembly, then the C2 bench with phase
# timings, then the C3 mscan / hashed-scan A/B.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-c2}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -k "c2 or c1 or parallel or pipelined or exact_walk or full_size or wide or multi_term or datetime or hit_list" --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 2 --tickets 100000 --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c2.json 2> gpurun_out/${T}_c2.err || { echo C2_FAIL; tail -20 gpurun_out/${T}_c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_c2.json'));r=d['roofline'];print('C2',d['value']/1e6,d['p50_ms'],r['kernel'],r['avg_launch_ms'],r['frac'])"
grep "pass" gpurun_out/${T}_c2.err | tail -2 | cut -c1-300
bash tools/gpu_ab_mhash_c3.sh ${T}m
