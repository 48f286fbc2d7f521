# Round 4 (session 2): marker-scene parity probe, the fused residual-add LayerNorm forward A/B against
# lib_prev (two processes back to back), the bench line, a kernel-stats profile of a short bench run and
# every GPU test.  First failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r04f}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pose.py tests/test_gpu_layernorm.py tests/test_gpu_attention.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$OUT/pytest_pose.log 2>&1 || { echo PYTEST POSE FAILED; tail -30 gpurun_out/$OUT/pytest_pose.log; exit 1; }
tail -1 gpurun_out/$OUT/pytest_pose.log
timeout -k 10 500 python3 -u tools/parity3d_probe.py --frames 24 --seeds 7 > gpurun_out/$OUT/parity3d.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/$OUT/parity3d.log; exit 1; }
grep "^{" gpurun_out/$OUT/parity3d.log
timeout -k 10 300 python3 -u tools/vit_probe.py --knob 12=1 --iters 10 --rounds 3 > gpurun_out/$OUT/probe_new.log 2>&1 || { echo PROBE FAILED; tail -20 gpurun_out/$OUT/probe_new.log; exit 1; }
timeout -k 10 300 python3 -u tools/vit_probe.py --lib macaque-3d-pose-estimation_amd/lib_prev/libmq_hip.so --knob 12=1 --iters 10 --rounds 3 > gpurun_out/$OUT/probe_prev.log 2>&1 || { echo PROBE PREV FAILED; tail -20 gpurun_out/$OUT/probe_prev.log; exit 1; }
grep -h "ms per forward" gpurun_out/$OUT/probe_new.log gpurun_out/$OUT/probe_prev.log
timeout -k 10 600 python3 bench.py > gpurun_out/$OUT/bench.json 2> gpurun_out/$OUT/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/$OUT/bench.err; exit 1; }
cut -c1-600 gpurun_out/$OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --no-cpu-baseline --no-lift --no-config5 --no-extras > gpurun_out/$OUT/prof_bench.json 2> gpurun_out/$OUT/prof.err || { echo PROF FAILED; tail -20 gpurun_out/$OUT/prof.err; exit 1; }
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|Error" gpurun_out/$OUT/pytest_gpu.log | head; tail -30 gpurun_out/$OUT/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$OUT/pytest_gpu.log
