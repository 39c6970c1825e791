# Diagnostic A/B of mscan_kernel's dispatch-event duration in the C3 pass:
# candidates per lane (NKM_MSCAN_J) and n identical back-to-back launches
# before the timed one (NKM_MSCAN_WARM=n).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/warm.txt
for v in "NKM_MSCAN_J=2" "NKM_MSCAN_J=1" "NKM_MSCAN_J=1 NKM_MSCAN_WARM=4" "NKM_MSCAN_J=2 NKM_MSCAN_WARM=4" "NKM_MSCAN_J=1" "NKM_MSCAN_J=2"; do
  env $v timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/warm_x.json 2> gpurun_out/warm_x.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/warm_x.json')); r=d['roofline']
print('$v', 'mscan us', round(r['avg_launch_ms']*1e3,2), 'frac', round(r['frac'],3), 'p50', round(d['p50_ms'],2))" >> gpurun_out/warm.txt
done
echo EXIT $?
