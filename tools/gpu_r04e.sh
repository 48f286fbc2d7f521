# Round 4 batch: attention ring variant A/B (tests + isolated + forward), the one-wave-per-SIMD GEMM
# prototype, then the parity / clip3 / config3 checks of gpu_r04c.sh.  First failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r04e}
mkdir -p gpurun_out/$OUT
bash tools/gpu_ab_attention.sh $OUT || exit 1
timeout -k 10 300 python3 -u tools/proto/probe_w1.py --iters 20 --rounds 3 > gpurun_out/$OUT/proto_w1.log 2>&1 || { echo PROTO FAILED; tail -30 gpurun_out/$OUT/proto_w1.log; exit 1; }
cat gpurun_out/$OUT/proto_w1.log
bash tools/gpu_r04c.sh $OUT
