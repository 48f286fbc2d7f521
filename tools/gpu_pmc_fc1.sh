# rocprofv3 PMC passes (usage: gpu_pmc_fc1.sh <out> [pp|w4]) over the fc1 GEMM (gemm_pp_kernel<1, 0, 8, 4>: GELU epilogue, GEMM mode, 256x256 tiles) of the ViT-H bench shape, one counter
# group per pass (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass), then the
# per-launch summary with the gfx950 corrections -> gpurun_out/$OUT/pmc_fc1_gemm.json.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-pmc}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python3 -c "import torch" || exit 1
i=0
VAR=${2:-pp}
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/gemm_probe.py --iters 5 --shape fc1 --variants $VAR > gpurun_out/$OUT/p$i.log 2>&1 || { echo "PMC pass $i ($grp) failed"; tail -5 gpurun_out/$OUT/p$i.log; exit 1; }
  echo "PMC pass $i ($grp) ok"
done
KNAME="gemm_pp_kernel<1, 0, 8, 4>"
[ "$VAR" = "w4" ] && KNAME="gemm_w4_kernel<1, false>"
python3 tools/pmc_summary.py gpurun_out/$OUT "$KNAME" 170414080 161061273600 > gpurun_out/$OUT/pmc_fc1_gemm.json
head -40 gpurun_out/$OUT/pmc_fc1_gemm.json
