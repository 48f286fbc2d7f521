# RCCL rehearsal of bench.py's N > 1 code on a one-GPU box: one rank under torch.distributed.run with the
# nccl (RCCL) backend and MQ_BENCH_DIST=1, so the process group, the barriers, the keypoint all-gather on
# device tensors, the max-over-ranks timing and the clip lift of the gathered keypoints all run.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-rccl}
mkdir -p gpurun_out/$OUT
MQ_BENCH_DIST=1 NCCL_DEBUG=INFO NCCL_DEBUG_FILE=$GRAFT_REPO_ROOT/gpurun_out/$OUT/nccl.%p.txt timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
  --no-config5 --no-extras > gpurun_out/$OUT/bench.json 2> gpurun_out/$OUT/bench.err || { echo BENCH FAILED; tail -30 gpurun_out/$OUT/bench.err; exit 1; }
cat gpurun_out/$OUT/bench.json
grep -h -i "rccl version\|Init COMPLETE" gpurun_out/$OUT/nccl.*.txt || true
# the config-3 clip driver's sharded step 1 with its all-gather over RCCL (one rank, process group forced)
MQ_DIST_FORCE=1 NCCL_DEBUG=INFO NCCL_DEBUG_FILE=$GRAFT_REPO_ROOT/gpurun_out/$OUT/nccl_clip.%p.txt timeout -k 10 600 \
  python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29518 \
  tools/run_clip_sharded.py --root /tmp/mq_clip3r --sharded > gpurun_out/$OUT/clip3_rccl.json 2> gpurun_out/$OUT/clip3_rccl.err || { echo CLIP3 RCCL FAILED; tail -30 gpurun_out/$OUT/clip3_rccl.err; exit 1; }
cat gpurun_out/$OUT/clip3_rccl.json
grep -h -i "AllGather\|Init COMPLETE" gpurun_out/$OUT/nccl_clip.*.txt | head -5 || true
