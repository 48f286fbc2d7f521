# The rest of r04s after its lift A/B stopped on lib_base's older ABI: config-4 lift (lib, then lib_base), the
# parity probe at seeds 8 and 9 with the ABI-6 solver defaults, then the RCCL world-1 rehearsal (bench N > 1
# path and the config-3 clip's after-gather time).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r04t}
L=macaque-3d-pose-estimation_amd
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python3 -u tools/lift_probe.py --reps 5 > gpurun_out/$OUT/lift_new.json 2> gpurun_out/$OUT/lift_new.err || { echo LIFT NEW FAILED; tail -20 gpurun_out/$OUT/lift_new.err; exit 1; }
timeout -k 10 300 python3 -u tools/lift_probe.py --lib $L/lib_base/libmq_hip.so --reps 5 > gpurun_out/$OUT/lift_base.json 2> gpurun_out/$OUT/lift_base.err || { echo LIFT BASE FAILED; tail -20 gpurun_out/$OUT/lift_base.err; exit 1; }
cut -c1-420 gpurun_out/$OUT/lift_new.json gpurun_out/$OUT/lift_base.json
timeout -k 10 600 python3 -u tools/parity3d_probe.py --frames 24 --seeds 8,9 > gpurun_out/$OUT/parity3d.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/$OUT/parity3d.log; exit 1; }
grep '"n_frames": 24' gpurun_out/$OUT/parity3d.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print(json.dumps({k: v for k, v in d.items() if k.startswith(('solver', 'scipy', 'optim', 'kp3d_optim', 'kp3d_dlt_mm_all', 'kp_max', 'clear', 'argmax', 'seed'))}))"
bash tools/gpu_rccl_rehearsal.sh $OUT
