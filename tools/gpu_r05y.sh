# Round 5: contiguous hashed scan with 2 candidates per lane — the chunk-shape
# and proven-list tests, mhash_bench, and the C3 / C4 lines with
# NKM_MCONTIG_J=2 vs the default 4, interleaved.  $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05y}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "chunk_lengths or proven_mscan or counts_only" > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^FAILED|Error|assert" gpurun_out/${T}_tests.log | head -30; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 180 tools/mhash_bench > gpurun_out/${T}_mhash_bench.txt 2>&1 || { echo MHB_FAIL; tail -20 gpurun_out/${T}_mhash_bench.txt; exit 1; }
grep -E "count dbg 0" gpurun_out/${T}_mhash_bench.txt
for k in 3_4a 3_2a 4_4a 4_2a 3_4b 3_2b 4_4b 4_2b; do
  C=${k:0:1}; J=${k:2:1}
  NKM_MCONTIG_J=$J timeout -k 10 300 python bench.py --config $C --steps 10 --no-cpu-baseline > gpurun_out/${T}_c$k.json 2> gpurun_out/${T}_c$k.err || { echo BENCH_FAIL; tail -20 gpurun_out/${T}_c$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c$k.json').read().strip().splitlines()[-1]); r=d['roofline']
print('c$k', round(d['value']/1e6, 2), 'M/s p50', round(d['p50_ms'], 2), r.get('kernel'), round(r['avg_launch_ms']*1e3, 2), 'us frac', round(r['frac'], 3))"
done
