# LayerNorm A/B: the LayerNorm GPU test on the candidate build, then mq_layernorm timed in one process
# for lib_prev vs lib and lib_prev vs lib_rpw4 (bit-identity checked), then the ViT-H forward of both builds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-ab_ln}
mkdir -p gpurun_out/$OUT
L=macaque-3d-pose-estimation_amd
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_layernorm.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/$OUT/pytest.log; exit 1; }
tail -2 gpurun_out/$OUT/pytest.log
timeout -k 10 300 python3 -u tools/ab_gemm.py --a $L/lib_prev/libmq_hip.so --b $L/lib/libmq_hip.so --shape "" --layernorm --iters 50 --rounds 3 > gpurun_out/$OUT/ab2.log 2>&1 || { echo AB FAILED; tail -20 gpurun_out/$OUT/ab2.log; exit 1; }
cat gpurun_out/$OUT/ab2.log
if [ -f $L/lib_rpw4/libmq_hip.so ]; then
  timeout -k 10 300 python3 -u tools/ab_gemm.py --a $L/lib_prev/libmq_hip.so --b $L/lib_rpw4/libmq_hip.so --shape "" --layernorm --iters 50 --rounds 3 > gpurun_out/$OUT/ab4.log 2>&1 || { echo AB4 FAILED; tail -20 gpurun_out/$OUT/ab4.log; exit 1; }
  cat gpurun_out/$OUT/ab4.log
fi
