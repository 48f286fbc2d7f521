# Round 3, first GPU pass over the new paths: config-2 batch parity, the config-5 frame graph, config 3
# end to end (single process, world-1 sharded, 2 ranks on one GPU), then the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r03a}
mkdir -p gpurun_out/$OUT
timeout -k 10 1500 python3 -u -m pytest tests/test_gpu_attention.py tests/test_gpu_frame_graph.py \
  "tests/test_gpu_pose.py::test_vitpose_h_config2_batch_vs_fp32_oracle" tests/test_gpu_config3.py \
  -m gpu -v -rA --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|Error" gpurun_out/$OUT/pytest_gpu.log | head -20; tail -40 gpurun_out/$OUT/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/$OUT/pytest_gpu.log
timeout -k 10 900 python3 bench.py > gpurun_out/$OUT/bench.json 2> gpurun_out/$OUT/bench.err || { echo BENCH FAILED; tail -30 gpurun_out/$OUT/bench.err; exit 1; }
cat gpurun_out/$OUT/bench.json
