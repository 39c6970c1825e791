# Full -m gpu suite + smoke + C3/C4/C5 lines on the split pass sources,
# then the 2-rank gloo rehearsal (tools/gpu_dist_r03.sh).  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r03n}
bash tools/gpu_r03l.sh $T && bash tools/gpu_dist_r03.sh ${T}d
