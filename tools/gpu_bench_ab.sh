# bench.py under several MQ_TUNING settings ($2: ';'-separated, "-" = defaults), interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-bab}
mkdir -p gpurun_out/$OUT
IFS=';' read -ra CFGS <<< "${2:--}"
for r in 0 1; do
for c in "${CFGS[@]}"; do
  t=""; [ "$c" != "-" ] && t="$c"
  MQ_TUNING="$t" timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps ${3:-20} > gpurun_out/$OUT/b.json 2> gpurun_out/$OUT/b.err || { echo BENCH FAILED "$c"; tail -20 gpurun_out/$OUT/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/$OUT/b.json'));print('r$r', '$c', d['value'], d['ms_per_step'], d['roofline']['achieved'])"
done
done
