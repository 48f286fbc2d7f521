# PMC passes on the attention kernel (attn_probe, all modes; summarise mode-0 dispatches offline).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/apmc
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE" "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/apmc/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/attn_probe.py > gpurun_out/apmc/p$i.log 2>&1 || { echo PMC $i FAILED; tail -20 gpurun_out/apmc/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob
from collections import defaultdict
vals = defaultdict(list)
for f in sorted(glob.glob("gpurun_out/apmc/p*/run_counter_collection.csv")):
    rows = [r for r in csv.DictReader(open(f)) if "attention2_kernel<80, 192>" in r["Kernel_Name"]]
    for r in rows:
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(vals.items()):
    print(k, len(v), sum(v) / len(v))
PY
