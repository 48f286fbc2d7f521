# ABI 6 (optim_points stop test at ftol / 2, two steps in a row) + the PCG latency work: the optim / pipeline /
# parity / run_demo / config-3 GPU tests, the config-4 lift against lib_base, the parity probe at seeds 8 and 9,
# then the RCCL world-1 rehearsal (bench N > 1 path and the config-3 clip's after-gather time).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r04s}
L=macaque-3d-pose-estimation_amd
mkdir -p gpurun_out/$OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_optim.py tests/test_gpu_pipeline.py tests/test_gpu_parity3d.py tests/test_gpu_run_demo.py tests/test_gpu_config3.py -m gpu -x -v -s --timeout 800 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|Error|^E " gpurun_out/$OUT/pytest.log | cut -c1-400 | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/$OUT/pytest.log | tail -1
grep -E "parity3d {" gpurun_out/$OUT/pytest.log | cut -c1-1500
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
