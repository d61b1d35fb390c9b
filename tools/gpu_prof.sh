#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench per config, with the per-kernel summary and one
# iteration's launch timeline: bash tools/gpu_prof.sh TAG "cfg1 cfg2" [steps]
TAG=${1:?tag}; CFGS=${2:-ex10}; S=${3:-6}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for C in $CFGS; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$C -o run -- python3 bench.py --config $C --steps $S --warmup 1 --no-cpu --no-opt --legs none > $OUT/prof_$C.log 2>&1 \
    || { echo "$C rocprof FAILED"; tail -20 $OUT/prof_$C.log; exit 1; }
  python3 tools/prof_summary.py $OUT/prof_$C > $OUT/${C}_prof_summary.txt 2>&1
  python3 tools/iter_timeline.py $OUT/prof_$C > $OUT/${C}_iter_timeline.txt 2>&1
  echo "== $C"; head -16 $OUT/${C}_prof_summary.txt; tail -1 $OUT/${C}_iter_timeline.txt
done
