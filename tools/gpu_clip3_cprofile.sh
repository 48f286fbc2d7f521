# Where the config-3 clip driver's step 1 spends its time: cProfile of tools/run_clip_sharded.py at world 1
# (sharded path, no process group), top functions by cumulative and by own time.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-clip3prof}
mkdir -p gpurun_out/$OUT
timeout -k 10 300 python3 tools/run_clip_sharded.py --root /tmp/mq_clip3p --sharded > gpurun_out/$OUT/warm.json 2> gpurun_out/$OUT/warm.err || { echo WARM FAILED; tail -20 gpurun_out/$OUT/warm.err; exit 1; }
timeout -k 10 400 python3 -m cProfile -o gpurun_out/$OUT/clip.prof tools/run_clip_sharded.py --root /tmp/mq_clip3p --results /tmp/mq_clip3p/res_prof --sharded > gpurun_out/$OUT/clip.json 2> gpurun_out/$OUT/clip.err || { echo PROF FAILED; tail -20 gpurun_out/$OUT/clip.err; exit 1; }
cat gpurun_out/$OUT/warm.json gpurun_out/$OUT/clip.json
python3 -c "
import pstats
p = pstats.Stats('gpurun_out/$OUT/clip.prof')
p.sort_stats('cumulative').print_stats(45)
p.sort_stats('tottime').print_stats(30)
" > gpurun_out/$OUT/pstats.txt
head -120 gpurun_out/$OUT/pstats.txt | tail -100
