# optim_points defaults of ABI 5 (40 PCG iterations, two-step stop): the optim / pipeline / parity GPU tests,
# the config-4 lift timing with its kernel profile.  First failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r04i}
mkdir -p gpurun_out/$OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_optim.py tests/test_gpu_pipeline.py tests/test_gpu_parity3d.py tests/test_gpu_run_demo.py tests/test_gpu_pose.py -m gpu -x -v -s --timeout 800 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|Error|^E " gpurun_out/$OUT/pytest.log | cut -c1-400 | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/$OUT/pytest.log | tail -1
grep -E "parity3d {|clear fraction|clear\+taylor" gpurun_out/$OUT/pytest.log | cut -c1-3000
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/proflift -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_lift.py --no-cpu --reps 2 > gpurun_out/$OUT/proflift.json 2> gpurun_out/$OUT/proflift.err || { echo PROF LIFT FAILED; tail -20 gpurun_out/$OUT/proflift.err; exit 1; }
cat gpurun_out/$OUT/proflift.json
