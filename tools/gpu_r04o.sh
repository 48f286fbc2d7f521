# optim_points PCG latency work: config-4 lift A/B (timing + result digest, bit-identity expected) of lib
# (everything: matvec loads up front, p.q reduced by the matvec's last block, precond staging before the
# done check, G / H / I blocks in registers, interleaved rz butterflies, the factor's smoothness couplings precomputed) against lib_base and the partial
# builds lib_pq / lib_pq2 / lib_pq3, the config-3 clip (step-4 solver calls logged), the optim GPU tests,
# then the lift's kernel profile.  First failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r04o}
L=macaque-3d-pose-estimation_amd
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python3 -u tools/lift_probe.py --reps 5 > gpurun_out/$OUT/lift_new.json 2> gpurun_out/$OUT/lift_new.err || { echo LIFT NEW FAILED; tail -20 gpurun_out/$OUT/lift_new.err; exit 1; }
timeout -k 10 300 python3 -u tools/lift_probe.py --lib $L/lib_base/libmq_hip.so --reps 5 > gpurun_out/$OUT/lift_base.json 2> gpurun_out/$OUT/lift_base.err || { echo LIFT BASE FAILED; tail -20 gpurun_out/$OUT/lift_base.err; exit 1; }
timeout -k 10 300 python3 -u tools/lift_probe.py --lib $L/lib_pq/libmq_hip.so --reps 5 > gpurun_out/$OUT/lift_pq.json 2> gpurun_out/$OUT/lift_pq.err || { echo LIFT PQ FAILED; tail -20 gpurun_out/$OUT/lift_pq.err; exit 1; }
timeout -k 10 300 python3 -u tools/lift_probe.py --lib $L/lib_pq2/libmq_hip.so --reps 5 > gpurun_out/$OUT/lift_pq2.json 2> gpurun_out/$OUT/lift_pq2.err || { echo LIFT PQ2 FAILED; tail -20 gpurun_out/$OUT/lift_pq2.err; exit 1; }
timeout -k 10 300 python3 -u tools/lift_probe.py --lib $L/lib_pq3/libmq_hip.so --reps 5 > gpurun_out/$OUT/lift_pq3.json 2> gpurun_out/$OUT/lift_pq3.err || { echo LIFT PQ3 FAILED; tail -20 gpurun_out/$OUT/lift_pq3.err; exit 1; }
cut -c1-400 gpurun_out/$OUT/lift_new.json gpurun_out/$OUT/lift_base.json gpurun_out/$OUT/lift_pq.json gpurun_out/$OUT/lift_pq2.json gpurun_out/$OUT/lift_pq3.json
timeout -k 10 600 python3 -u tools/run_clip_sharded.py --root /tmp/mq_clip3 > gpurun_out/$OUT/clip3.json 2> gpurun_out/$OUT/clip3.err || { echo CLIP3 FAILED; tail -30 gpurun_out/$OUT/clip3.err; exit 1; }
cut -c1-3000 gpurun_out/$OUT/clip3.json
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_optim.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|^E " gpurun_out/$OUT/pytest.log | cut -c1-300 | head -20; exit 1; }
tail -1 gpurun_out/$OUT/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/proflift -o run -- python3 $GRAFT_REPO_ROOT/tools/lift_probe.py --reps 2 > gpurun_out/$OUT/proflift.json 2> gpurun_out/$OUT/proflift.err || { echo PROF LIFT FAILED; tail -20 gpurun_out/$OUT/proflift.err; exit 1; }
python3 tools/prof_summary.py $(find gpurun_out/$OUT/proflift -name "*kernel_stats.csv" | head -1) 1 14
