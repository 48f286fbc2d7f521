# Round 4 (session 2): the end-to-end parity probe on the marker scene (DLT propagation, optim vs scipy),
# PMC passes over the ViT-H forward after the residual move (proj = gemm_pp_kernel<0> launches 97:3:1, the
# fused add + LayerNorm kernels, attention), then the config-3 clip.  First failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r04g}
mkdir -p gpurun_out/$OUT
timeout -k 10 700 python3 -u tools/parity3d_probe.py --frames 24 --seeds 7 > gpurun_out/$OUT/parity3d.log 2>&1 || { echo PARITY PROBE FAILED; tail -30 gpurun_out/$OUT/parity3d.log; exit 1; }
grep "^{" gpurun_out/$OUT/parity3d.log
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/pmc/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/vit_probe.py --iters 2 --rounds 1 --knob 20=1 > gpurun_out/$OUT/pmc_p$i.log 2>&1 || { echo "PMC pass $i ($grp) failed"; tail -5 gpurun_out/$OUT/pmc_p$i.log; exit 1; }
  echo "PMC pass $i ($grp) ok"
done
# proj: A 31.46 MB + W 3.28 MB + out bf16 31.46 MB = 66.19 MB; 40.27 GFLOP
python3 tools/pmc_summary.py gpurun_out/$OUT/pmc "gemm_pp_kernel<0, 0, 8, 4>" 66191360 40265318400 97:3:1 > gpurun_out/$OUT/pmc_proj_gemm.json
# fc2: A 125.83 MB + W 13.11 MB + out bf16 31.46 MB = 170.41 MB; 161.06 GFLOP
python3 tools/pmc_summary.py gpurun_out/$OUT/pmc "gemm_pp_kernel<0, 0, 8, 4>" 170393600 161061273600 97:3:2 > gpurun_out/$OUT/pmc_fc2_gemm.json
# fused LN1 (x += p1 + p2, x stored, y): 62.91 + 2 x 31.46 + 62.91 + 31.46 MB = 220.2 MB
python3 tools/pmc_summary.py gpurun_out/$OUT/pmc "layernorm_kernel<5, false, 2, true>" 220200960 0 > gpurun_out/$OUT/pmc_add_ln1.json
# fused LN2 (x + p1 not stored, y): 62.91 + 31.46 + 31.46 MB = 125.8 MB
python3 tools/pmc_summary.py gpurun_out/$OUT/pmc "layernorm_kernel<5, false, 1, false>" 125829120 0 > gpurun_out/$OUT/pmc_add_ln2.json
python3 tools/pmc_summary.py gpurun_out/$OUT/pmc "attention2_kernel<80, 192>" 125829120 12079595520 > gpurun_out/$OUT/pmc_attention.json
python3 tools/pmc_summary.py gpurun_out/$OUT/pmc "gemm_pp_kernel<1, 0, 8, 4>" 170414080 161061273600 > gpurun_out/$OUT/pmc_fc1_gemm.json
for f in proj_gemm fc2_gemm add_ln1 add_ln2 attention fc1_gemm; do python3 -c "
import json,sys; d=json.load(open('gpurun_out/$OUT/pmc_$f.json'))
print('$f', {k: round(d[k],3) if isinstance(d.get(k),float) else d.get(k) for k in ('traffic_over_algorithmic','hbm_bytes_per_launch','l2_hit_rate','mfma_busy_per_gui_cycle','avg_duration_ns_under_pmc')})"; done
bash tools/gpu_clip3.sh $OUT || exit 1
