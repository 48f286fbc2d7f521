set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03a
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_detector.py::test_implicit_conv3x3_equals_im2col_gemm tests/test_gpu_pose.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03a/pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/r03a/pytest.log; exit 1; }
tail -2 gpurun_out/r03a/pytest.log
timeout -k 10 300 python3 -u tools/ab_gemm.py --a macaque-3d-pose-estimation_amd/lib_prev/libmq_hip.so --b macaque-3d-pose-estimation_amd/lib/libmq_hip.so --shape qkv,fc1,dc1,dc2,fc1_bf16 --iters 20 --rounds 3 > gpurun_out/r03a/ab.log 2>&1 || { echo AB FAILED; tail -30 gpurun_out/r03a/ab.log; exit 1; }
cat gpurun_out/r03a/ab.log
