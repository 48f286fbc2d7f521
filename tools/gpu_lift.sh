# Lift development call: optim / Viterbi GPU tests, the PCG-cap probe, a rocprof profile of the lift.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-lift}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_optim.py tests/test_gpu_geometry.py tests/test_gpu_pipeline.py -m gpu -x -q -rA --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|Error" gpurun_out/$OUT/pytest.log | head; tail -30 gpurun_out/$OUT/pytest.log; exit 1; }
tail -1 gpurun_out/$OUT/pytest.log
timeout -k 10 400 python3 -u tools/optim_probe.py > gpurun_out/$OUT/optim_probe.log 2>&1 || { echo PROBE FAILED; tail -20 gpurun_out/$OUT/optim_probe.log; exit 1; }
grep -v "^{" gpurun_out/$OUT/optim_probe.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/proflift -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_lift.py --no-cpu --reps 2 > gpurun_out/$OUT/proflift.json 2> gpurun_out/$OUT/proflift.err || { echo PROF LIFT FAILED; tail -20 gpurun_out/$OUT/proflift.err; exit 1; }
cat gpurun_out/$OUT/proflift.json
