set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-attn2}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_attention.py tests/test_gpu_pose.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/$OUT/pytest.log; exit 1; }
tail -1 gpurun_out/$OUT/pytest.log
timeout -k 10 200 python3 tools/attn_probe.py > gpurun_out/$OUT/attn_probe.txt 2>&1 || { echo ATTN PROBE FAILED; tail -20 gpurun_out/$OUT/attn_probe.txt; exit 1; }
grep "r=1" gpurun_out/$OUT/attn_probe.txt
for c in "15=0" "15=1" "15=0" "15=1"; do
  MQ_TUNING="$c" timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 20 > gpurun_out/$OUT/b.json 2> gpurun_out/$OUT/b.err || { echo BENCH FAILED "$c"; tail -20 gpurun_out/$OUT/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/$OUT/b.json'));print('bench', '$c', d['value'], d['ms_per_step'], d['roofline']['achieved'])"
done
