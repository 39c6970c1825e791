# Same-box A/B of host-side variants of the C3 pass: each line of $NKM_AB is
# "label ENV=VAL ..." ; runs are interleaved twice to expose box drift.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab.txt
for rep in 1 2; do
while IFS= read -r line; do
  [ -z "$line" ] && continue
  set -- $line
  label=$1; shift
  env "$@" NKM_PROFILE=1 timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$label.json 2> gpurun_out/ab_$label.err || exit 1
  python - "$label" >> gpurun_out/ab.txt <<'PY'
import json, sys, re
lab = sys.argv[1]
d = json.load(open(f"gpurun_out/ab_{lab}.json"))
ph = [l for l in open(f"gpurun_out/ab_{lab}.err") if l.startswith("[nkm]")]
def avg(key):
    v = [float(m.group(1)) for l in ph for m in [re.search(key + r" ([0-9.]+)", l)] if m]
    return sum(v) / len(v) if v else float("nan")
print(f"{lab:12s} {d['value']/1e6:6.1f} M/s p50 {d['p50_ms']:6.2f} | pass {avg('pass'):6.2f} replay {avg('replay'):6.2f} work {avg('work'):6.2f} taskmax {avg('task max'):6.2f} merge {avg('merge'):5.2f} finish {avg('finish'):5.2f}")
PY
done <<< "$NKM_AB"
done
echo EXIT $?
