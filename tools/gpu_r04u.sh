# Round 4 (session 2) final check, part 1: every GPU test at HEAD (ABI 6).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r04u}
mkdir -p gpurun_out/$OUT
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -v -rA --timeout 600 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|^E " gpurun_out/$OUT/pytest_gpu.log | cut -c1-300 | head -20; tail -3 gpurun_out/$OUT/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$OUT/pytest_gpu.log
