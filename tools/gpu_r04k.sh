# Detector residual updates through mq_add_layernorm: the LayerNorm / detector / frame-graph GPU tests, the
# detector timing (eager + graph) with its kernel summary.  First failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r04k}
mkdir -p gpurun_out/$OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_layernorm.py tests/test_gpu_detector.py tests/test_gpu_frame_graph.py -m gpu -x -q -rA --timeout 600 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|^E " gpurun_out/$OUT/pytest.log | cut -c1-300 | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/$OUT/pytest.log | tail -1
bash tools/gpu_det.sh $OUT
