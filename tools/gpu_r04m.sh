# GELU through the LDS table (gemm_pp / gemm256 epilogues): fc1 A/B against lib_base (HEAD before it) in one
# process, the GEMM / pose GPU tests, the ViT-H forward of both builds, then the multi-rank rehearsals.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r04m}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python3 -u tools/ab_gemm.py --a macaque-3d-pose-estimation_amd/lib_base/libmq_hip.so --b macaque-3d-pose-estimation_amd/lib/libmq_hip.so --shape fc1,fc1_bf16,qkv --iters 20 --rounds 3 > gpurun_out/$OUT/ab_fc1.log 2>&1 || { echo AB FAILED; tail -20 gpurun_out/$OUT/ab_fc1.log; exit 1; }
grep -v amdgpu.ids gpurun_out/$OUT/ab_fc1.log
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_pose.py tests/test_gpu_detector.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|^E " gpurun_out/$OUT/pytest.log | cut -c1-300 | head -20; exit 1; }
tail -1 gpurun_out/$OUT/pytest.log
timeout -k 10 300 python3 -u tools/vit_probe.py --knob 12=1 --iters 10 --rounds 3 > gpurun_out/$OUT/probe_new.log 2>&1 || { echo PROBE FAILED; tail -20 gpurun_out/$OUT/probe_new.log; exit 1; }
timeout -k 10 300 python3 -u tools/vit_probe.py --lib macaque-3d-pose-estimation_amd/lib_base/libmq_hip.so --knob 12=1 --iters 10 --rounds 3 > gpurun_out/$OUT/probe_base.log 2>&1 || { echo PROBE BASE FAILED; tail -20 gpurun_out/$OUT/probe_base.log; exit 1; }
grep -h "ms per forward" gpurun_out/$OUT/probe_new.log gpurun_out/$OUT/probe_base.log
bash tools/gpu_r04l.sh $OUT
