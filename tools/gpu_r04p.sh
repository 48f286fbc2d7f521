# r04q (streaming add + LayerNorm A/B), r04o (optim matvec / eval loads up front: lift A/B, config-3 clip, optim
# tests, lift profile), then the parity-3D probe at seeds 8 and 9 (r04n).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=${1:-r04p}
bash tools/gpu_r04q.sh $OUT && bash tools/gpu_r04o.sh $OUT && bash tools/gpu_r04n.sh $OUT
