# Round 4 (session 2) final check, part 2: smoke(), the default bench line (N=1), a rocprof kernel-stats
# profile of a short bench run.  First failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r04v}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$OUT/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/$OUT/smoke.log; exit 1; }
tail -1 gpurun_out/$OUT/smoke.log
timeout -k 10 900 python3 bench.py > gpurun_out/$OUT/bench.json 2> gpurun_out/$OUT/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/$OUT/bench.err; exit 1; }
cut -c1-900 gpurun_out/$OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --no-cpu-baseline --no-lift --no-config5 --no-extras > gpurun_out/$OUT/prof_bench.json 2> gpurun_out/$OUT/prof.err || { echo PROF FAILED; tail -20 gpurun_out/$OUT/prof.err; exit 1; }
echo PROF OK
