# Development GPU call: selected GPU tests, then optional probes (attention, GEMM).
# usage: gpu_dev.sh OUTDIR "pytest -k expr or ''" "probe list: attn gemm bench" [test paths...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$1; K=$2; PROBES=$3
shift 3
PATHS=${@:-tests}
mkdir -p gpurun_out/$OUT
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python3 -u -m pytest $PATHS -m gpu -x -q -rA --timeout 240 --timeout-method thread "${KARG[@]}" > gpurun_out/$OUT/pytest_gpu.log 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|Error|error" gpurun_out/$OUT/pytest_gpu.log | head -30; tail -30 gpurun_out/$OUT/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$OUT/pytest_gpu.log
for p in $PROBES; do
  case $p in
    attn) timeout -k 10 300 python3 tools/attn_probe.py > gpurun_out/$OUT/attn_probe.log 2>&1 || { echo ATTN PROBE FAILED; tail -20 gpurun_out/$OUT/attn_probe.log; exit 1; }; cat gpurun_out/$OUT/attn_probe.log ;;
    gemm) timeout -k 10 300 python3 tools/gemm_probe.py --iters 20 --shape qkv,proj,fc1,fc2,dc1,dc2 --variants pp,il,torch > gpurun_out/$OUT/gemm_probe.log 2>&1 || { echo GEMM PROBE FAILED; tail -20 gpurun_out/$OUT/gemm_probe.log; exit 1; }; grep " r=1" gpurun_out/$OUT/gemm_probe.log ;;
    bench) timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/$OUT/bench.json 2> gpurun_out/$OUT/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/$OUT/bench.err; exit 1; }; cat gpurun_out/$OUT/bench.json ;;
  esac
done
