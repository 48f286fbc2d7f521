# GEMM tests (all 256x256 variants) + probe of variants on the ViT shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tune
timeout -k 10 300 python3 -m pytest tests/test_gpu_gemm.py -m gpu -x -q > gpurun_out/tune/pytest_gemm.log 2>&1 || { echo GEMM TESTS FAILED; tail -30 gpurun_out/tune/pytest_gemm.log; exit 1; }
tail -2 gpurun_out/tune/pytest_gemm.log
timeout -k 10 600 python3 tools/gemm_probe.py --iters 20 --shape qkv,proj,fc1,fc2,dc1,dc2,f32,n5120_k5120 --variants ${1:-4,buf4,m32,bm32,torch} > gpurun_out/tune/probe.txt 2>&1 || { echo PROBE FAILED; tail -30 gpurun_out/tune/probe.txt; exit 1; }
grep -v "^{" gpurun_out/tune/probe.txt | grep "r=1"
