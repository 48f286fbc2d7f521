# optim_points vs scipy on the marker-scene oracle chain's 2D (tools/optim_parity_probe.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-r04h}
mkdir -p gpurun_out/$OUT
timeout -k 10 900 python3 -u tools/optim_parity_probe.py --frames 24 --pcg 20,40 --stop 0,1,2,3 --ftol 1e-3 > gpurun_out/$OUT/optim_probe.log 2>&1 || { echo PROBE FAILED; tail -30 gpurun_out/$OUT/optim_probe.log; exit 1; }
grep "^{" gpurun_out/$OUT/optim_probe.log
