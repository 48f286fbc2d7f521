set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03y
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03y/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_detector.py --steps 1 > gpurun_out/r03y/det.log 2>&1 || { tail -20 gpurun_out/r03y/det.log; exit 1; }
ls gpurun_out/r03y/prof
