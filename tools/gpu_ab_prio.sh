set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03y
L=macaque-3d-pose-estimation_amd
for v in ${VARIANTS:-p1 p2}; do
  timeout -k 10 300 python3 -u tools/ab_gemm.py --a $L/lib_prev/libmq_hip.so --b $L/lib_$v/libmq_hip.so --shape qkv,fc1,fc2,dc1 --iters 20 --rounds 3 > gpurun_out/r03y/ab_$v.log 2>&1 || { echo AB $v FAILED; tail -20 gpurun_out/r03y/ab_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/r03y/ab_$v.log
done
[ -n "$TRACE" ] && bash tools/gpu_det_trace.sh; true
