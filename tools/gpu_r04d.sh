# Round 4: one-wave-per-SIMD GEMM prototype A/B against the ping-pong kernel, then gpu_r04c.sh.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r04d}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python3 -u tools/proto/probe_w1.py --iters 20 --rounds 3 > gpurun_out/$OUT/proto_w1.log 2>&1 || { echo PROTO FAILED; tail -30 gpurun_out/$OUT/proto_w1.log; exit 1; }
cat gpurun_out/$OUT/proto_w1.log
bash tools/gpu_r04c.sh $OUT
