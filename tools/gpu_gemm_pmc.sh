# GEMM probe timings + rocprofv3 PMC passes on the fc1-shaped GEMM (one pass per counter group).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/gemm_probe.py --iters 20 > gpurun_out/pmc/probe.txt 2>&1; echo "PROBE $?"; cat gpurun_out/pmc/probe.txt | grep -v "^{"
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1; echo "LIST $?"
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS" "GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/gemm_probe.py --iters 3 --shape fc1 > gpurun_out/pmc/p$i.log 2>&1
  echo "PMC $i ($grp) exit $?"
done
