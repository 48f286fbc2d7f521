set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r06b}; mkdir -p gpurun_out/$OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_gemm_w4.py -x -v --timeout 200 --timeout-method thread > gpurun_out/$OUT/t.log 2>&1 || { echo TEST FAILED; tail -40 gpurun_out/$OUT/t.log; exit 1; }
tail -3 gpurun_out/$OUT/t.log
timeout -k 10 300 python3 -u tools/gemm_probe.py --shape qkv,proj_bf16,fc1,fc2_bf16,dc1 --variants pp,w4,w4v --iters 20 > gpurun_out/$OUT/probe.log 2>&1 || { echo PROBE FAILED; tail -30 gpurun_out/$OUT/probe.log; exit 1; }
grep " v=" gpurun_out/$OUT/probe.log
