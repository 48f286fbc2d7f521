# One GPU call: GPU tests, bench (N=1), rocprof kernel stats of the bench, GEMM probe vs torch.
# Each GPU step has its own time limit; the first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-chk}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/$OUT/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/$OUT/pytest_gpu.log
timeout -k 10 400 python3 bench.py > gpurun_out/$OUT/bench.json 2> gpurun_out/$OUT/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/$OUT/bench.err; exit 1; }
cat gpurun_out/$OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --no-cpu-baseline > gpurun_out/$OUT/prof_bench.json 2> gpurun_out/$OUT/prof.err || { echo PROF FAILED; tail -20 gpurun_out/$OUT/prof.err; exit 1; }
timeout -k 10 300 python3 tools/gemm_probe.py --iters 20 --variants 4,torch > gpurun_out/$OUT/gemm_probe.log 2>&1 || { echo PROBE FAILED; tail -20 gpurun_out/$OUT/gemm_probe.log; exit 1; }
grep " r=1" gpurun_out/$OUT/gemm_probe.log
