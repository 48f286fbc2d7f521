# Full round check: every GPU test, smoke(), the default bench line (N=1), a rocprofv3 kernel-stats
# profile of a short bench run, then the fc1 PMC passes.  First failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-full}
TESTS=${2:-tests}   # pytest paths (default: every GPU test)
mkdir -p gpurun_out/$OUT
timeout -k 10 1200 python3 -u -m pytest $TESTS -m gpu -v -rA --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|Error" gpurun_out/$OUT/pytest_gpu.log | head; tail -30 gpurun_out/$OUT/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$OUT/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/$OUT/smoke.log; exit 1; }
tail -1 gpurun_out/$OUT/smoke.log
timeout -k 10 600 python3 bench.py > gpurun_out/$OUT/bench.json 2> gpurun_out/$OUT/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/$OUT/bench.err; exit 1; }
cat gpurun_out/$OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --no-cpu-baseline --no-lift --no-config5 --no-extras > gpurun_out/$OUT/prof_bench.json 2> gpurun_out/$OUT/prof.err || { echo PROF FAILED; tail -20 gpurun_out/$OUT/prof.err; exit 1; }
for fps in 2 4; do  # multi-frame batches (bench multi_frame_batches.fps2 / fps4): their own kernel stats
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/prof_fps$fps -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --frames-per-step $fps --no-cpu-baseline --no-lift --no-config5 --no-extras > gpurun_out/$OUT/prof_fps$fps.json 2> gpurun_out/$OUT/prof_fps$fps.err || { echo PROF FPS$fps FAILED; tail -20 gpurun_out/$OUT/prof_fps$fps.err; exit 1; }
done
bash tools/gpu_pmc_fc1.sh $OUT/pmc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/proflift -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_lift.py --no-cpu --reps 2 > gpurun_out/$OUT/proflift.json 2> gpurun_out/$OUT/proflift.err || { echo PROF LIFT FAILED; tail -20 gpurun_out/$OUT/proflift.err; exit 1; }
cat gpurun_out/$OUT/proflift.json
# config 3 (the clip driver) runs in its own call: tools/gpu_clip3.sh
