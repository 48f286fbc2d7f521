# Round 4: the end-to-end 2D -> 3D parity probe (tools/parity3d_probe.py), the config-3 clip through the
# camera-sharded tail (world 1 sharded, then 2 ranks sharing the GPU over gloo), and the GPU tests touched.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r04c}
mkdir -p gpurun_out/$OUT
timeout -k 10 500 python3 -u tools/parity3d_probe.py --frames 24 --seeds 7 > gpurun_out/$OUT/parity3d.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/$OUT/parity3d.log; exit 1; }
cat gpurun_out/$OUT/parity3d.log
bash tools/gpu_clip3.sh $OUT || exit 1
timeout -k 10 900 python3 -u -m pytest -x -v -s --timeout 900 --timeout-method thread tests/test_gpu_config3.py tests/test_gpu_pipeline.py > gpurun_out/$OUT/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/$OUT/pytest.log; grep "timings" gpurun_out/$OUT/pytest.log
exit $rc
