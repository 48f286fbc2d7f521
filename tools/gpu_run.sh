#!/bin/bash
# One parameterised runner for the GPU box (replaces the per-round gpu_r0*.sh batch scripts):
#   gpurun -- 'bash tools/gpu_run.sh <out> <step> [<step> ...]'
# Each step runs under its own time limit, writes gpurun_out/<out>/<step>.log, and the first failing step
# ends the run (no GPU step after a fault).  Steps:
#   tests[:<pytest args>]  pytest -m gpu (all GPU tests, or the given files / -k expression)
#   smoke                  __graft_entry__.smoke()
#   bench[:<args>]         python bench.py <args>  (JSON line -> <out>/bench.json)
#   bench2[:<args>]        bench.py as 2 ranks sharing the one GPU over gloo (MQ_BENCH_SHARE_GPU=1): a rehearsal
#                          of the multi-rank path (gather, max-over-ranks, the split clip lift)
#   prof[:<args>]          rocprofv3 --kernel-trace --stats over bench.py <args> -> <out>/prof/
#   tool:<script> [args]   python tools/<script> <args>
#   profpy:<script> [args] rocprofv3 --kernel-trace --stats over python tools/<script>
set -o pipefail
out=gpurun_out/$1
shift
mkdir -p "$out"
export TMPDIR=/tmp
run() {  # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  echo "[gpu_run] $name: $*"
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "[gpu_run] $name rc=$rc"
  tail -3 "$out/$name.log"
  return $rc
}
i=0
for step in "$@"; do
  i=$((i + 1))
  kind=${step%%:*}
  arg=""
  [[ "$step" == *:* ]] && arg=${step#*:}
  case $kind in
    tests) run "t$i" 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${arg:-tests} || exit $? ;;
    smoke) run "smoke$i" 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) run "bench$i" 900 python -u bench.py $arg || exit $?
           grep '^{' "$out/bench$i.log" | tail -1 > "$out/bench$i.json" ;;
    bench2) run "bench2_$i" 900 env MQ_BENCH_SHARE_GPU=1 MQ_BENCH_BACKEND=gloo python -u -m torch.distributed.run --nnodes=1 \
              --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29540 + i)) bench.py --gpus 2 $arg || exit $?
            grep '^{' "$out/bench2_$i.log" | tail -1 > "$out/bench2_$i.json" ;;
    prof) run "prof$i" 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof$i" -o run -- python3 -u bench.py $arg || exit $? ;;
    tool) run "tool$i" 900 python -u tools/$arg || exit $? ;;
    profpy) run "profpy$i" 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/profpy$i" -o run -- python3 -u tools/$arg || exit $? ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
