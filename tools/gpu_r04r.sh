# optim_points PCG latency work without the fused p.q reduction (matvec loads up front, precond staging before
# the done check, G / H / I blocks in registers, interleaved rz butterflies, factor couplings precomputed,
# recurrence unrolled by 2): config-4 lift A/B against lib_base (timing + result digest, bit-identity
# expected), the lift's kernel profile, the optim / pipeline GPU tests, the config-3 clip (step-4 solver
# calls logged), then the solver against scipy on the marker scenes of seeds 7, 8, 9 at three ftol values.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r04r}
L=macaque-3d-pose-estimation_amd
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python3 -u tools/lift_probe.py --reps 5 > gpurun_out/$OUT/lift_new.json 2> gpurun_out/$OUT/lift_new.err || { echo LIFT NEW FAILED; tail -20 gpurun_out/$OUT/lift_new.err; exit 1; }
timeout -k 10 300 python3 -u tools/lift_probe.py --lib $L/lib_base/libmq_hip.so --reps 5 > gpurun_out/$OUT/lift_base.json 2> gpurun_out/$OUT/lift_base.err || { echo LIFT BASE FAILED; tail -20 gpurun_out/$OUT/lift_base.err; exit 1; }
cut -c1-330 gpurun_out/$OUT/lift_new.json gpurun_out/$OUT/lift_base.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/proflift -o run -- python3 $GRAFT_REPO_ROOT/tools/lift_probe.py --reps 2 > gpurun_out/$OUT/proflift.json 2> gpurun_out/$OUT/proflift.err || { echo PROF LIFT FAILED; tail -20 gpurun_out/$OUT/proflift.err; exit 1; }
python3 tools/prof_summary.py $(find gpurun_out/$OUT/proflift -name "*kernel_stats.csv" | head -1) 1 8
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_optim.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|^E " gpurun_out/$OUT/pytest.log | cut -c1-300 | head -20; exit 1; }
tail -1 gpurun_out/$OUT/pytest.log
timeout -k 10 600 python3 -u tools/run_clip_sharded.py --root /tmp/mq_clip3 > gpurun_out/$OUT/clip3.json 2> gpurun_out/$OUT/clip3.err || { echo CLIP3 FAILED; tail -30 gpurun_out/$OUT/clip3.err; exit 1; }
cut -c1-1200 gpurun_out/$OUT/clip3.json
timeout -k 10 700 python3 -u tools/optim_parity_probe.py --frames 24 --seeds 7,8,9 --pcg 40 --stop 2 --ftol 1e-3,5e-4,2.5e-4 > gpurun_out/$OUT/solver_probe.log 2>&1 || { echo SOLVER PROBE FAILED; tail -30 gpurun_out/$OUT/solver_probe.log; exit 1; }
grep "^{" gpurun_out/$OUT/solver_probe.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); d.pop('rows', None); print(json.dumps(d))"
