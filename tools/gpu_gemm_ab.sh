# GEMM numerics tests + GEMM probe A/B (variants given as $2) + bench.  First failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-ab}
VARS=${2:-4,b256}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$OUT/pytest_gemm.log 2>&1 || { echo GEMM TESTS FAILED; tail -30 gpurun_out/$OUT/pytest_gemm.log; exit 1; }
tail -2 gpurun_out/$OUT/pytest_gemm.log
timeout -k 10 300 python3 tools/gemm_probe.py --iters 20 --shape ${3:-qkv,proj,fc1,fc2,dc1,dc2} --variants $VARS > gpurun_out/$OUT/gemm_probe.log 2>&1 || { echo PROBE FAILED; tail -20 gpurun_out/$OUT/gemm_probe.log; exit 1; }
grep " r=1" gpurun_out/$OUT/gemm_probe.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/$OUT/bench.json 2> gpurun_out/$OUT/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/$OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/$OUT/bench.json'));print('BENCH', d['value'], d['ms_per_step'], d['roofline']['achieved'])"
