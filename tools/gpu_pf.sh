set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-pf}
mkdir -p gpurun_out/$OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/$OUT/pytest.log; exit 1; }
tail -1 gpurun_out/$OUT/pytest.log
timeout -k 10 300 python3 tools/gemm_probe.py --iters 20 --shape proj,fc2 --variants pp,pf0 > gpurun_out/$OUT/gemm_probe.log 2>&1 || { echo PROBE FAILED; tail -20 gpurun_out/$OUT/gemm_probe.log; exit 1; }
grep " r=1" gpurun_out/$OUT/gemm_probe.log
for c in "16=0" "16=1" "16=0" "16=1"; do
  MQ_TUNING="$c" timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 20 > gpurun_out/$OUT/b.json 2> gpurun_out/$OUT/b.err || { echo BENCH FAILED "$c"; tail -20 gpurun_out/$OUT/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/$OUT/b.json'));print('bench', '$c', d['value'], d['ms_per_step'], d['roofline']['achieved'])"
done
