# trust-region solver with 5 frames per workgroup (config 4: 240 workgroups, one round) against 4 (300): GPU tests of
# the solver and the step-4 pipeline, then optim_points timing at both settings in one process each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-trf_fb}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_optim_trf.py tests/test_gpu_optim.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$OUT/t.log 2>&1 || { echo TEST FAILED; tail -30 gpurun_out/$OUT/t.log; exit 1; }
tail -2 gpurun_out/$OUT/t.log
timeout -k 10 300 python3 -u tools/optim_solver_timing.py --solvers trf --cases config4 --fb 4 > gpurun_out/$OUT/fb4.log 2>&1 || { echo FB4 FAILED; tail -20 gpurun_out/$OUT/fb4.log; exit 1; }
timeout -k 10 300 python3 -u tools/optim_solver_timing.py --solvers trf --cases config4 --fb 5 > gpurun_out/$OUT/fb5.log 2>&1 || { echo FB5 FAILED; tail -20 gpurun_out/$OUT/fb5.log; exit 1; }
timeout -k 10 300 python3 -u tools/optim_solver_timing.py --solvers trf --cases config4 --fb 4 > gpurun_out/$OUT/fb4b.log 2>&1 || { echo FB4b FAILED; tail -20 gpurun_out/$OUT/fb4b.log; exit 1; }
grep -h '^{' gpurun_out/$OUT/fb4.log gpurun_out/$OUT/fb5.log gpurun_out/$OUT/fb4b.log
