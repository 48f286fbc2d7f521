# BASELINE config 3 end to end on one GPU: the clip driver through the sharded path at world 1, then as
# 2 ranks sharing the GPU over gloo.  First failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-clip3}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 python3 tools/run_clip_sharded.py --root /tmp/mq_clip3 --sharded > gpurun_out/$OUT/clip3_world1.json 2> gpurun_out/$OUT/clip3_world1.err || { echo CLIP3 FAILED; tail -20 gpurun_out/$OUT/clip3_world1.err; exit 1; }
cat gpurun_out/$OUT/clip3_world1.json
MQ_DIST_BACKEND=gloo MQ_SHARE_GPU=1 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/run_clip_sharded.py --root /tmp/mq_clip3 --results /tmp/mq_clip3/res2 > gpurun_out/$OUT/clip3_world2_gloo.json 2> gpurun_out/$OUT/clip3_world2_gloo.err || { echo CLIP3 W2 FAILED; tail -20 gpurun_out/$OUT/clip3_world2_gloo.err; exit 1; }
cat gpurun_out/$OUT/clip3_world2_gloo.json
