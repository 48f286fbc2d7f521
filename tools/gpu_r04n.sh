# Parity-3D statements on more scenes: the marker-scene probe at seeds 8 and 9 (config 2 + a 24-frame slice).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r04n}
mkdir -p gpurun_out/$OUT
timeout -k 10 900 python3 -u tools/parity3d_probe.py --frames 24 --seeds 8,9 > gpurun_out/$OUT/parity3d.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/$OUT/parity3d.log; exit 1; }
grep "^{" gpurun_out/$OUT/parity3d.log
