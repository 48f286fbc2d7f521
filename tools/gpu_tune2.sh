# GEMM + attention tests, GEMM variant probe, hipBLASLt kernel names.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tune2
timeout -k 10 300 python3 -m pytest tests/test_gpu_gemm.py tests/test_gpu_pose.py -m gpu -x -q > gpurun_out/tune2/pytest.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/tune2/pytest.log; exit 1; }
tail -2 gpurun_out/tune2/pytest.log
timeout -k 10 600 python3 tools/gemm_probe.py --iters 20 --shape qkv,proj,fc1,fc2,dc1,dc2,n5120_k5120 --variants buf4,sch > gpurun_out/tune2/probe.txt 2>&1 || { echo PROBE FAILED; tail -30 gpurun_out/tune2/probe.txt; exit 1; }
grep -v "^{" gpurun_out/tune2/probe.txt | grep "r=1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tune2/tn -o run -- python3 $GRAFT_REPO_ROOT/tools/gemm_probe.py --iters 5 --shape qkv,proj,fc1,fc2,dc1,n5120_k5120 --variants torch > gpurun_out/tune2/tn.txt 2>&1 || { echo TN FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tune2/bp -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --no-cpu-baseline > gpurun_out/tune2/bench.json 2> gpurun_out/tune2/bench.err || { echo BENCH FAILED; tail -5 gpurun_out/tune2/bench.err; exit 1; }
cat gpurun_out/tune2/bench.json
