# Kernel names/durations hipBLASLt picks for the ViT GEMM shapes (torch.matmul), for tile-shape reference.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tnames
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tnames -o run -- python3 $GRAFT_REPO_ROOT/tools/gemm_probe.py --iters 5 --shape qkv,proj,fc1,fc2,dc1,n5120_k5120 --variants torch > gpurun_out/tnames/probe.txt 2>&1 || { echo FAILED; tail -20 gpurun_out/tnames/probe.txt; exit 1; }
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/tnames/run_kernel_stats.csv")))
for r in rows:
    if "Cijk" in r["Name"] or "gemm" in r["Name"].lower():
        print(r["Calls"], round(float(r["AverageNs"]) / 1000, 2), r["Name"][:400])
PY
