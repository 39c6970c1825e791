# GPU parity tests, then same-box A/B of mscan_kernel with and without the
# order[] indirection (NKM_DIRECT), interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
: > gpurun_out/direct_ab.txt
for rep in 1 2; do
  for d in 0 1; do
    NKM_DIRECT=$d timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/direct_$d.json 2> gpurun_out/direct_$d.err || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/direct_$d.json')); r=d['roofline']
print('NKM_DIRECT=$d', round(d['value']/1e6,1), 'M/s p50', round(d['p50_ms'],2), 'mscan us', round(r['avg_launch_ms']*1e3,2), 'bytes', r['bytes_per_launch'], 'frac', round(r['frac'],3))" >> gpurun_out/direct_ab.txt
  done
done
echo EXIT $?
