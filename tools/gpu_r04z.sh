# factor recurrence with the next frame's LDS inputs read ahead (lib_fp) against HEAD
# (lib): config-4 lift timing and result digest (bit-identity expected), alternating, then lib_fp's kernel profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r04z}
L=macaque-3d-pose-estimation_amd
mkdir -p gpurun_out/$OUT
for r in 1 2; do
  timeout -k 10 300 python3 -u tools/lift_probe.py --lib $L/lib_fp/libmq_hip.so --reps 5 > gpurun_out/$OUT/lift_fp$r.json 2> gpurun_out/$OUT/lift_fp$r.err || { echo LIFT MV FAILED; tail -20 gpurun_out/$OUT/lift_fp$r.err; exit 1; }
  timeout -k 10 300 python3 -u tools/lift_probe.py --reps 5 > gpurun_out/$OUT/lift_head$r.json 2> gpurun_out/$OUT/lift_head$r.err || { echo LIFT HEAD FAILED; tail -20 gpurun_out/$OUT/lift_head$r.err; exit 1; }
done
cut -c1-300 gpurun_out/$OUT/lift_fp1.json gpurun_out/$OUT/lift_head1.json gpurun_out/$OUT/lift_fp2.json gpurun_out/$OUT/lift_head2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/proflift -o run -- python3 $GRAFT_REPO_ROOT/tools/lift_probe.py --lib $GRAFT_REPO_ROOT/$L/lib_fp/libmq_hip.so --reps 2 > gpurun_out/$OUT/proflift.json 2> gpurun_out/$OUT/proflift.err || { echo PROF LIFT FAILED; tail -20 gpurun_out/$OUT/proflift.err; exit 1; }
python3 tools/prof_summary.py $(find gpurun_out/$OUT/proflift -name "*kernel_stats.csv" | head -1) 1 6
