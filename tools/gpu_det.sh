# Detector timing (eager + graph) and its rocprof kernel summary -> gpurun_out/$1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-det}
mkdir -p gpurun_out/$OUT
timeout -k 10 400 python3 -u tools/bench_detector.py --steps 10 --graph > gpurun_out/$OUT/bench_det.json 2> gpurun_out/$OUT/bench_det.err || { tail -20 gpurun_out/$OUT/bench_det.err; exit 1; }
cat gpurun_out/$OUT/bench_det.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$OUT/prof -o run -- python3 tools/bench_detector.py --steps 3 > gpurun_out/$OUT/prof.log 2>&1 || { tail -20 gpurun_out/$OUT/prof.log; exit 1; }
f=$(ls gpurun_out/$OUT/prof/*kernel_stats.csv | head -1); python3 tools/prof_summary.py $f 5 30
