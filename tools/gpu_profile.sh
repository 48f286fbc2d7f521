# rocprofv3 kernel-trace + stats of a short bench run (ROCm 7.2).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${1:-prof}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$OUT -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$OUT.bench.json 2> gpurun_out/$OUT.err
echo "PROF EXIT $?"
find gpurun_out/$OUT -name "*stats*" | head
