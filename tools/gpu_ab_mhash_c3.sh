# Same-box A/B on the C3 headline: mscan_kernel (default, 8 signatures) vs
# the hashed scan (NKM_MHASH=1: cuckoo lookup, contiguous vector loads with
# 4 or 8 candidates per lane), interleaved, with the eval kernel's duration
# and frac per run.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-abm}
for R in 1 2; do
  for V in "NKM_MHASH=0" "NKM_MHASH=1" "NKM_MHASH=1 NKM_MCONTIG_J=8"; do
    N=$(echo $V | tr -d ' =_')
    env $V timeout -k 10 300 python bench.py --steps 11 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_${N}_$R.json 2> gpurun_out/${T}_${N}_$R.err || { echo "FAIL $V"; tail -20 gpurun_out/${T}_${N}_$R.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${T}_${N}_$R.json'));r=d['roofline'];print('$V',round(d['value']/1e6,1),round(d['p50_ms'],3),r['kernel'],round(r['avg_launch_ms']*1e3,2),'us',round(r['frac'],3))"
  done
done
