# Ping-pong GEMM timing ablations on the bf16-epilogue shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-ppabl}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python3 tools/gemm_probe.py --iters 20 --shape ${3:-qkv,dc1,fc1_bf16} --variants ${2:-pp,pa1,pa2,pa3,pa4,pa8,pa15} > gpurun_out/$OUT/gemm_probe.log 2>&1 || { echo PROBE FAILED; tail -20 gpurun_out/$OUT/gemm_probe.log; exit 1; }
grep " r=1" gpurun_out/$OUT/gemm_probe.log
