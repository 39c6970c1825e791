# The hashed scan in isolation (tools/mhash_bench: one-chunk-per-workgroup vs
# the resident pipelined loop, counts-only; C4 4M / 64 sigs and C3 1M / 8),
# then SQ counter passes over the same program (one counter group per run).
# $1 = tag.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05d}
timeout -k 10 120 tools/mhash_bench > gpurun_out/${T}_mhash_bench.txt 2>&1 || { echo MHB_FAIL; tail -20 gpurun_out/${T}_mhash_bench.txt; exit 1; }
grep -E "cldW|lists" gpurun_out/${T}_mhash_bench.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_mhb_trace -o run -- tools/mhash_bench > gpurun_out/${T}_mhb_trace.log 2>&1 || { echo TRACE_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/${T}_mhb_sq1 -o sq -- tools/mhash_bench > gpurun_out/${T}_mhb_sq1.log 2>&1 || { echo SQ1_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_mhb_sq2 -o sq -- tools/mhash_bench > gpurun_out/${T}_mhb_sq2.log 2>&1 || { echo SQ2_FAIL; exit 1; }
echo DONE
