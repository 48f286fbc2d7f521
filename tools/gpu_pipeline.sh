# GPU tests of optim_points + the drop-in pipeline entry points.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -m pytest tests/test_gpu_pipeline.py tests/test_gpu_optim.py -m gpu -x -q -rA > gpurun_out/pytest_pipeline.log 2>&1
rc=$?; echo "PYTEST EXIT $rc"; tail -40 gpurun_out/pytest_pipeline.log; exit $rc
