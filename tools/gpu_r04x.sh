# HEAD after the matvec preload: the optim / pipeline / parity / config-3 GPU tests and smoke().
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r04x}
mkdir -p gpurun_out/$OUT
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_optim.py tests/test_gpu_pipeline.py tests/test_gpu_parity3d.py tests/test_gpu_config3.py tests/test_gpu_run_demo.py -m gpu -v -rA --timeout 600 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|^E " gpurun_out/$OUT/pytest.log | cut -c1-300 | head -20; exit 1; }
tail -1 gpurun_out/$OUT/pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$OUT/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/$OUT/smoke.log; exit 1; }
tail -1 gpurun_out/$OUT/smoke.log
