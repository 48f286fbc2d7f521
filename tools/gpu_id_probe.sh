# 64x64-tile GEMM check: GEMM / ID / detector GPU tests, the ID forward A/B (tile64 on / off), a rocprof
# kernel-stats pass of the 13-box ID forward.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r03f}
mkdir -p gpurun_out/$OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_resnet_id.py tests/test_gpu_gemm.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/$OUT/pytest.log; exit 1; }
tail -2 gpurun_out/$OUT/pytest.log
timeout -k 10 300 python3 -u tools/id_probe.py 13 32 > gpurun_out/$OUT/id_probe.log 2>&1 || { echo PROBE FAILED; tail -20 gpurun_out/$OUT/id_probe.log; exit 1; }
cat gpurun_out/$OUT/id_probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/id_probe.py 13 > gpurun_out/$OUT/prof.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/$OUT/prof.log; exit 1; }
head -12 gpurun_out/$OUT/prof/run_kernel_stats.csv | cut -c1-160
