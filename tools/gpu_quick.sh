# Pose/GEMM GPU tests + bench (no CPU baseline) + kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-quick}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python3 -m pytest tests/test_gpu_gemm.py tests/test_gpu_pose.py -m gpu -x -q > gpurun_out/$OUT/pytest.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/$OUT/pytest.log; exit 1; }
tail -2 gpurun_out/$OUT/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/bp -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --no-cpu-baseline > gpurun_out/$OUT/bench.json 2> gpurun_out/$OUT/bench.err || { echo BENCH FAILED; tail -5 gpurun_out/$OUT/bench.err; exit 1; }
cat gpurun_out/$OUT/bench.json
python3 - <<PY
import csv
rows = list(csv.DictReader(open("gpurun_out/$OUT/bp/run_kernel_stats.csv")))
for r in rows[:8]:
    print(r["Calls"], round(float(r["AverageNs"]) / 1000, 2), r["Percentage"][:5], r["Name"][:90])
PY
