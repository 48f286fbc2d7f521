# Streaming fused add + LayerNorm (layernorm_stream_kernel, -DLN_STREAM, LN_STREAM_WAVES 1024 / 2048 / 4096):
# mq_add_layernorm A/B against lib_base at the bench rows (64 images x 192 tokens) (bit-identity expected), then the ViT-H
# forward of lib_base and lib_ln2048.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r04q}
L=macaque-3d-pose-estimation_amd
mkdir -p gpurun_out/$OUT
for v in 2048 1024 4096; do
  timeout -k 10 200 python3 -u tools/ab_gemm.py --a $L/lib_base/libmq_hip.so --b $L/lib_ln$v/libmq_hip.so --shape "" --add-layernorm --iters 20 --rounds 3 > gpurun_out/$OUT/ab_ln$v.log 2>&1 || { echo AB $v FAILED; tail -20 gpurun_out/$OUT/ab_ln$v.log; exit 1; }
  echo "== waves $v"; grep -v amdgpu.ids gpurun_out/$OUT/ab_ln$v.log
done
timeout -k 10 300 python3 -u tools/vit_probe.py --lib $L/lib_ln2048/libmq_hip.so --knob 12=1 --iters 10 --rounds 3 > gpurun_out/$OUT/probe_ln2048.log 2>&1 || { echo PROBE FAILED; tail -20 gpurun_out/$OUT/probe_ln2048.log; exit 1; }
timeout -k 10 300 python3 -u tools/vit_probe.py --lib $L/lib_base/libmq_hip.so --knob 12=1 --iters 10 --rounds 3 > gpurun_out/$OUT/probe_base.log 2>&1 || { echo PROBE BASE FAILED; tail -20 gpurun_out/$OUT/probe_base.log; exit 1; }
grep -h "ms per forward" gpurun_out/$OUT/probe_ln2048.log gpurun_out/$OUT/probe_base.log
