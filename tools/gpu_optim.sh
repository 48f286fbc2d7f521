# GPU optim_points parity tests only.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -m pytest tests/test_gpu_optim.py -m gpu -x -q -rA > gpurun_out/pytest_optim.log 2>&1
rc=$?; echo "PYTEST EXIT $rc"; tail -30 gpurun_out/pytest_optim.log; exit $rc
