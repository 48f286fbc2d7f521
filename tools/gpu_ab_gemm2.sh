# GEMM A/B against lib_prev: the GEMM / pose GPU tests on this build, ab_gemm on the ViT-H shapes (both
# builds in one process), the ViT-H forward of both builds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$1
mkdir -p gpurun_out/$OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_pose.py tests/test_gpu_deconv.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/$OUT/pytest.log; exit 1; }
tail -2 gpurun_out/$OUT/pytest.log
timeout -k 10 300 python3 -u tools/ab_gemm.py --a macaque-3d-pose-estimation_amd/lib_prev/libmq_hip.so --b macaque-3d-pose-estimation_amd/lib/libmq_hip.so --shape qkv,fc1,fc2,dc1,fc1_bf16 --iters 20 --rounds 3 > gpurun_out/$OUT/ab_gemm.log 2>&1 || { echo AB FAILED; tail -20 gpurun_out/$OUT/ab_gemm.log; exit 1; }
grep -v amdgpu.ids gpurun_out/$OUT/ab_gemm.log
timeout -k 10 300 python3 -u tools/vit_probe.py --knob 12=1 --iters 10 --rounds 3 > gpurun_out/$OUT/probe_new.log 2>&1 || { echo PROBE FAILED; tail -20 gpurun_out/$OUT/probe_new.log; exit 1; }
timeout -k 10 300 python3 -u tools/vit_probe.py --lib macaque-3d-pose-estimation_amd/lib_prev/libmq_hip.so --knob 12=1 --iters 10 --rounds 3 > gpurun_out/$OUT/probe_prev.log 2>&1 || { echo PROBE PREV FAILED; tail -20 gpurun_out/$OUT/probe_prev.log; exit 1; }
grep -h "ms per forward" gpurun_out/$OUT/probe_new.log gpurun_out/$OUT/probe_prev.log
