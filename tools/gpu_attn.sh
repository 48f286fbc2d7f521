set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/attn
timeout -k 10 300 python3 -m pytest tests/test_gpu_attention.py tests/test_gpu_pose.py -m gpu -x -q > gpurun_out/attn/pytest.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/attn/pytest.log; exit 1; }
tail -2 gpurun_out/attn/pytest.log
timeout -k 10 300 python3 tools/attn_probe.py > gpurun_out/attn/probe.txt 2>&1 || { echo PROBE FAILED; tail -20 gpurun_out/attn/probe.txt; exit 1; }
cat gpurun_out/attn/probe.txt
