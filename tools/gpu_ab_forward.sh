# Forward A/B against the previous build: pose / detector / attention GPU tests, the ViT-H forward of this build
# and of lib_prev (two processes back to back on one box), a short bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-ab_fwd}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pose.py tests/test_gpu_detector.py tests/test_gpu_attention.py tests/test_gpu_run_demo.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/$OUT/pytest.log; exit 1; }
tail -2 gpurun_out/$OUT/pytest.log
timeout -k 10 300 python3 -u tools/ab_gemm.py --a macaque-3d-pose-estimation_amd/lib_prev/libmq_hip.so --b macaque-3d-pose-estimation_amd/lib/libmq_hip.so --shape qkv --attention --iters 20 --rounds 3 > gpurun_out/$OUT/ab_attn.log 2>&1 && grep -i attention gpurun_out/$OUT/ab_attn.log && timeout -k 10 300 python3 -u tools/vit_probe.py --knob 12=1 --iters 10 --rounds 3 > gpurun_out/$OUT/probe_new.log 2>&1 || { echo PROBE FAILED; tail -20 gpurun_out/$OUT/probe_new.log; exit 1; }
timeout -k 10 300 python3 -u tools/vit_probe.py --lib macaque-3d-pose-estimation_amd/lib_prev/libmq_hip.so --knob 12=1 --iters 10 --rounds 3 > gpurun_out/$OUT/probe_prev.log 2>&1 || { echo PROBE PREV FAILED; tail -20 gpurun_out/$OUT/probe_prev.log; exit 1; }
grep -h "ms per forward" gpurun_out/$OUT/probe_new.log gpurun_out/$OUT/probe_prev.log
timeout -k 10 400 python3 bench.py --steps 50 --no-cpu-baseline --no-lift --no-config5 > gpurun_out/$OUT/bench.json 2> gpurun_out/$OUT/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/$OUT/bench.err; exit 1; }
cut -c1-400 gpurun_out/$OUT/bench.json
