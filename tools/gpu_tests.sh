# One GPU call: run the selected GPU tests (default: all) with per-test time limits.
# usage: gpu_tests.sh OUTDIR [pytest -k expression] [test paths...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-tests}
K=${2:-}
shift 2 2>/dev/null
PATHS=${@:-tests}
mkdir -p gpurun_out/$OUT
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python3 -u -m pytest $PATHS -m gpu -x -v -rA --timeout 240 --timeout-method thread "${KARG[@]}" > gpurun_out/$OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/$OUT/pytest_gpu.log | tail -40
exit $rc
