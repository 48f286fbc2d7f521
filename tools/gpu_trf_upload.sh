# optim_points' uploads as a mapped-memory kernel (lib/) against hipMemcpyAsync (lib_prev/): GPU tests of the solver and
# the step-4 pipeline on lib/, then config-4 / marker-scene timing alternating the two builds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-trf_upload}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_optim_trf.py tests/test_gpu_optim.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$OUT/t.log 2>&1 || { echo TEST FAILED; tail -30 gpurun_out/$OUT/t.log; exit 1; }
tail -2 gpurun_out/$OUT/t.log
for r in 1 2; do
  timeout -k 10 300 python3 -u tools/optim_solver_timing.py --solvers trf --cases config4,s7f24 --lib macaque-3d-pose-estimation_amd/lib_prev/libmq_hip.so > gpurun_out/$OUT/prev$r.log 2>&1 || { echo PREV FAILED; tail -20 gpurun_out/$OUT/prev$r.log; exit 1; }
  timeout -k 10 300 python3 -u tools/optim_solver_timing.py --solvers trf --cases config4,s7f24 > gpurun_out/$OUT/new$r.log 2>&1 || { echo NEW FAILED; tail -20 gpurun_out/$OUT/new$r.log; exit 1; }
done
for f in prev1 new1 prev2 new2; do echo $f; grep -h '^{' gpurun_out/$OUT/$f.log | cut -c1-160; done
