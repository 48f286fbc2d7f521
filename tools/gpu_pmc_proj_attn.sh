# rocprofv3 PMC passes over the ViT-H forward (tools/vit_probe.py, head-major QKV, 32 crops = 64 images),
# one counter group per pass, then per-launch summaries of the two kernels furthest from roofline:
#   proj      = gemm256_kernel<2>  (f32 residual epilogue, M 12288, N 1280, K 1280):
#               algorithmic bytes A 31.46 MB + W 3.28 MB + residual read + write 2 x 62.91 MB = 160.56 MB,
#               40.27 GFLOP per launch;
#   attention = attention2_kernel<80, 192> (64 images x 16 heads): Q, K, V read once 94.37 MB + O written
#               31.46 MB = 125.83 MB, 12.08 GFLOP per launch.
# Usage: bash tools/gpu_pmc_proj_attn.sh <out> [proj-kernel-substring] [attention-kernel-substring]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-pmc_pa}
PROJ=${2:-gemm256_kernel<2>}
ATTN=${3:-attention2_kernel<80, 192>}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python3 -c "import torch" || exit 1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/vit_probe.py --iters 2 --rounds 1 --knob 20=1 > gpurun_out/$OUT/p$i.log 2>&1 || { echo "PMC pass $i ($grp) failed"; tail -5 gpurun_out/$OUT/p$i.log; exit 1; }
  echo "PMC pass $i ($grp) ok"
done
python3 tools/pmc_summary.py gpurun_out/$OUT "$PROJ" 160563200 40265318400 > gpurun_out/$OUT/pmc_proj_gemm.json
python3 tools/pmc_summary.py gpurun_out/$OUT "$ATTN" 125829120 12079595520 > gpurun_out/$OUT/pmc_attention.json
head -50 gpurun_out/$OUT/pmc_proj_gemm.json gpurun_out/$OUT/pmc_attention.json
