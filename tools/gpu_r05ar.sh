# Round 5: contiguous count-only mscan_hash_kernel, 4 vs 8 candidates per lane
# (NKM_MCONTIG_J) on C4 4M and C3 1M — rocprofv3 kernel-trace averages and the
# bench's event timing, interleaved.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05ar}
for cfg in 4 3; do
  for k in a b; do
    for j in 4 8; do
      NKM_MCONTIG_J=$j timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c${cfg}_j$j$k -o run -- python3 bench.py --config $cfg --steps 8 --no-cpu-baseline > gpurun_out/${T}_c${cfg}_j$j$k.json 2> gpurun_out/${T}_c${cfg}_j$j$k.err || { echo PROF_FAIL; tail -20 gpurun_out/${T}_c${cfg}_j$j$k.err; exit 1; }
      python3 - "$cfg" "$j" "$k" "gpurun_out/${T}_c${cfg}_j$j$k" <<'PY'
import csv, json, sys
cfg, j, k, d = sys.argv[1:5]
rows = list(csv.DictReader(open(d + "/run_kernel_stats.csv")))
mh = [r for r in rows if "mscan_hash_kernel" in r["Name"]]
line = json.loads(open(d + ".json").read().strip().splitlines()[-1])
r = line["roofline"]
print(f"c{cfg} J{j} {k}: rocprof avg {float(mh[0]['AverageNs'])/1e3:.2f} us (min {float(mh[0]['MinNs'])/1e3:.2f}) | events {r['avg_launch_ms']*1e3:.2f} us frac {r['frac']:.3f} | {line['value']/1e6:.1f} M/s p50 {line['p50_ms']:.2f}")
PY
    done
  done
done
