# Pose / geometry GPU tests, the ViT-H forward under MQ_TUNE_GEMM_TILE64 (final 1x1 conv on 64x64 tiles)
# on / off in one process, and a short bench with the lift keys.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r03i}
mkdir -p gpurun_out/$OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_pose.py tests/test_gpu_geometry.py tests/test_gpu_pipeline.py tests/test_gpu_run_demo.py tests/test_gpu_gemm.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/$OUT/pytest.log; exit 1; }
tail -2 gpurun_out/$OUT/pytest.log
timeout -k 10 300 python3 -u tools/vit_probe.py --knob 19=1,0 --iters 10 --rounds 3 > gpurun_out/$OUT/probe.log 2>&1 || { echo PROBE FAILED; tail -20 gpurun_out/$OUT/probe.log; exit 1; }
grep "ms per" gpurun_out/$OUT/probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --no-cpu-baseline --no-lift --no-config5 > gpurun_out/$OUT/prof_bench.json 2> gpurun_out/$OUT/prof.err || { echo PROF FAILED; tail -20 gpurun_out/$OUT/prof.err; exit 1; }
grep -E "triangulate|undistort|gemm_bf16_kernel<5|col2im|decode|crop|flip" gpurun_out/$OUT/prof/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
