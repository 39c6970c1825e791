# Round 5 profiles: per-phase timings (NKM_PROFILE=2) of C3, C5, C2 and
# C5 + override, then PMC traffic of the C3 / C4 hashed scans (counts-only
# kernel), copied to profiles/r05_c{3,4}_traffic.json.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05f}
for C in 3 5 2; do
  NKM_PROFILE=2 timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_p2_c$C.json 2> gpurun_out/${T}_p2_c$C.err || { echo P2_FAIL $C; tail -20 gpurun_out/${T}_p2_c$C.err; exit 1; }
done
NKM_PROFILE=2 timeout -k 10 300 python bench.py --config 5 --override --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_p2_c5o.json 2> gpurun_out/${T}_p2_c5o.err || { echo P2_FAIL c5o; tail -20 gpurun_out/${T}_p2_c5o.err; exit 1; }
for C in 3 4; do
  bash tools/gpu_pmc_cfg.sh ${T}_c${C} $C mscan_hash_kernel || exit 1
  cat gpurun_out/${T}_c${C}_traffic.json; echo
done
