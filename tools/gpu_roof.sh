# The attainable duration of one mscan-sized launch (tools/mscan_roof.hip),
# then the GPU parity tests, smoke and a short headline bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/mscan_roof > gpurun_out/mscan_roof.txt 2>&1 && \
bash tools/gpu_tests.sh
