set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 -rA > gpurun_out/pytest_gpu2.log 2>&1; echo "PYTEST EXIT $?"; tail -25 gpurun_out/pytest_gpu2.log
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench2.json 2> gpurun_out/bench2.err; echo "BENCH EXIT $?"; cat gpurun_out/bench2.json; tail -5 gpurun_out/bench2.err
