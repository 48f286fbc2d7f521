# Small-tile GEMM A/B (gemm_bf16_kernel 64x64 / 128x128: the ID classifier and the detector's late
# stages): GEMM / ID / detector GPU tests on the candidate build (SKIP_TESTS=1: not), then the ID
# forward and the detector timed with lib_prev and lib (two processes each, back to back, alternating).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-ab_small}
mkdir -p gpurun_out/$OUT
P=macaque-3d-pose-estimation_amd/lib_prev/libmq_hip.so
N=macaque-3d-pose-estimation_amd/lib/libmq_hip.so
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_resnet_id.py tests/test_gpu_detector.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/$OUT/pytest.log; exit 1; }
  tail -2 gpurun_out/$OUT/pytest.log
fi
if [ -z "$SKIP_ID" ]; then
  for L in $P $N $P $N; do
    timeout -k 10 300 python3 -u tools/id_probe.py --lib $L 7 32 >> gpurun_out/$OUT/id.log 2>&1 || { echo ID PROBE FAILED; tail -20 gpurun_out/$OUT/id.log; exit 1; }
  done
  cat gpurun_out/$OUT/id.log
fi
for L in $P $N $P $N; do
  echo "== $L" >> gpurun_out/$OUT/det.log
  timeout -k 10 300 python3 -u tools/bench_detector.py --lib $L --steps 10 >> gpurun_out/$OUT/det.log 2>&1 || { echo DET FAILED; tail -20 gpurun_out/$OUT/det.log; exit 1; }
done
cat gpurun_out/$OUT/det.log
