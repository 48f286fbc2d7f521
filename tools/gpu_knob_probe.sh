# GPU tests of the forward path, then the ViT-H forward A/B under one same-result knob in one process.
# usage: bash tools/gpu_knob_probe.sh OUT KNOB=V1,V2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-knob}
KNOB=${2:-20=1,0}
mkdir -p gpurun_out/$OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_pose.py tests/test_gpu_attention.py tests/test_gpu_gemm.py tests/test_gpu_run_demo.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/$OUT/pytest.log; exit 1; }
tail -2 gpurun_out/$OUT/pytest.log
timeout -k 10 300 python3 -u tools/vit_probe.py --knob $KNOB --iters 10 --rounds 3 > gpurun_out/$OUT/probe.log 2>&1 || { echo PROBE FAILED; tail -20 gpurun_out/$OUT/probe.log; exit 1; }
grep "ms per" gpurun_out/$OUT/probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/vit_probe.py --knob $KNOB --iters 5 --rounds 1 > gpurun_out/$OUT/prof.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/$OUT/prof.log; exit 1; }
grep -E "attention|gemm_pp_kernel<0" gpurun_out/$OUT/prof/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
