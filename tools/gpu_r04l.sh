# Multi-rank rehearsals at HEAD on the one-GPU box: bench.py's N > 1 path over RCCL at world 1 and the config-3
# clip driver's all-gather over RCCL (tools/gpu_rccl_rehearsal.sh), then bench.py as 2 ranks sharing the GPU
# over gloo (n_gpus 2 in the JSON line; the value is still one GPU's aggregate).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r04l}
mkdir -p gpurun_out/$OUT
bash tools/gpu_rccl_rehearsal.sh $OUT || exit 1
MQ_BENCH_SHARE_GPU=1 MQ_BENCH_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-config5 \
  --no-extras > gpurun_out/$OUT/bench_2ranks_gloo.json 2> gpurun_out/$OUT/bench_2ranks_gloo.err || { echo BENCH 2 RANKS FAILED; tail -30 gpurun_out/$OUT/bench_2ranks_gloo.err; exit 1; }
cut -c1-600 gpurun_out/$OUT/bench_2ranks_gloo.json
