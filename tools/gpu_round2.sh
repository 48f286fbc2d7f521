# One GPU call: full GPU test suite, bench (N=1, with CPU baseline), rocprof kernel stats of the bench,
# PMC passes of the fc1 GEMM (ping-pong kernel).  Every GPU step has its own limit; first failure ends it.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r01e}
mkdir -p gpurun_out/$OUT/pmc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest_gpu.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/$OUT/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/$OUT/pytest_gpu.log
timeout -k 10 600 python3 bench.py > gpurun_out/$OUT/bench.json 2> gpurun_out/$OUT/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/$OUT/bench.err; exit 1; }
cat gpurun_out/$OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --no-cpu-baseline > gpurun_out/$OUT/prof_bench.json 2> gpurun_out/$OUT/prof.err || { echo PROF FAILED; tail -20 gpurun_out/$OUT/prof.err; exit 1; }
cat gpurun_out/$OUT/prof_bench.json
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/pmc/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/gemm_probe.py --iters 3 --shape fc1 --variants pp > gpurun_out/$OUT/pmc/p$i.log 2>&1 || { echo PMC $i FAILED; tail -20 gpurun_out/$OUT/pmc/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/$OUT/pmc "gemm_pp_kernel<1, 0>" 170414080 161061273600 > gpurun_out/$OUT/pmc_fc1_gemm.json
cat gpurun_out/$OUT/pmc_fc1_gemm.json
