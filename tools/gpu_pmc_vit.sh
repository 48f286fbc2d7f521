# rocprofv3 PMC passes over the ViT-H forward (tools/vit_probe.py: head-major QKV, 32 crops = 64 images), one counter
# group per pass, then per-launch summaries (tools/pmc_summary.py) of
#   attention = attention2_kernel<80, 192>: Q, K, V read once 94.37 MB + O written 31.46 MB = 125.83 MB,
#               12.08 GFLOP per launch;
#   fc1       = gemm_pp_kernel<1, 0, 8, 4> (GELU epilogue, M 12288 N 5120 K 1280) inside the forward:
#               A 31.46 + W 13.11 + C 125.83 MB = 170.41 MB, 161.06 GFLOP per launch.
# Usage: bash tools/gpu_pmc_vit.sh <out>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-pmc_vit}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python3 -c "import torch" || exit 1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/vit_probe.py --iters 2 --rounds 1 --knob 20=1 > gpurun_out/$OUT/p$i.log 2>&1 || { echo "PMC pass $i ($grp) failed"; tail -5 gpurun_out/$OUT/p$i.log; exit 1; }
  echo "PMC pass $i ($grp) ok"
done
python3 tools/pmc_summary.py gpurun_out/$OUT "attention2_kernel<80, 192>" 125829120 12079595520 > gpurun_out/$OUT/pmc_attention.json
python3 tools/pmc_summary.py gpurun_out/$OUT "gemm_pp_kernel<1, 0, 8, 4>" 170414080 161061273600 > gpurun_out/$OUT/pmc_fc1_in_forward.json
head -60 gpurun_out/$OUT/pmc_attention.json gpurun_out/$OUT/pmc_fc1_in_forward.json
