set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-ab}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_detector.py tests/test_gpu_pose.py tests/test_gpu_deconv.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/$OUT/pytest.log; exit 1; }
tail -2 gpurun_out/$OUT/pytest.log
timeout -k 10 300 python3 -u tools/ab_gemm.py --a macaque-3d-pose-estimation_amd/lib_prev/libmq_hip.so --b macaque-3d-pose-estimation_amd/lib/libmq_hip.so --shape qkv,proj,fc1,fc2,dc1,dc2 --iters 20 --rounds 3 > gpurun_out/$OUT/ab.log 2>&1 || { echo AB FAILED; tail -30 gpurun_out/$OUT/ab.log; exit 1; }
cat gpurun_out/$OUT/ab.log
