# optim_points / lift A/B: the optim and pipeline GPU tests on the in-tree library, then the config-4
# lift timed alternately with lib_prev (A) and lib (B), then a kernel-stats profile of B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-liftab}
mkdir -p gpurun_out/$OUT
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python3 -u -m pytest tests/test_gpu_optim.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/$OUT/pytest.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 gpurun_out/$OUT/pytest.log
for r in 0 1; do
  timeout -k 10 200 python3 tools/bench_lift.py --no-cpu --lib macaque-3d-pose-estimation_amd/lib_prev/libmq_hip.so > gpurun_out/$OUT/a$r.json 2> gpurun_out/$OUT/a$r.err || { echo A FAILED; tail -20 gpurun_out/$OUT/a$r.err; exit 1; }
  echo A$r; cat gpurun_out/$OUT/a$r.json
  timeout -k 10 200 python3 tools/bench_lift.py --no-cpu > gpurun_out/$OUT/b$r.json 2> gpurun_out/$OUT/b$r.err || { echo B FAILED; tail -20 gpurun_out/$OUT/b$r.err; exit 1; }
  echo B$r; cat gpurun_out/$OUT/b$r.json
  timeout -k 10 200 python3 tools/lift_probe.py --lib macaque-3d-pose-estimation_amd/lib_prev/libmq_hip.so > gpurun_out/$OUT/pa$r.json 2> gpurun_out/$OUT/pa$r.err || { echo PA FAILED; tail -20 gpurun_out/$OUT/pa$r.err; exit 1; }
  echo PA$r; cat gpurun_out/$OUT/pa$r.json
  timeout -k 10 200 python3 tools/lift_probe.py > gpurun_out/$OUT/pb$r.json 2> gpurun_out/$OUT/pb$r.err || { echo PB FAILED; tail -20 gpurun_out/$OUT/pb$r.err; exit 1; }
  echo PB$r; cat gpurun_out/$OUT/pb$r.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_lift.py --no-cpu --reps 2 > gpurun_out/$OUT/prof.json 2> gpurun_out/$OUT/prof.err || { echo PROF FAILED; tail -20 gpurun_out/$OUT/prof.err; exit 1; }
cat gpurun_out/$OUT/prof.json
