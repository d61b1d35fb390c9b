#!/bin/bash
# Focused GPU pass (run on the gpurun box from the repo root): a pytest selection, then the bench
# with an environment knob at each value (A/B), then the tree debug of the default.
# usage: KNOB=MADIPM_X VALUES="0 1" SEL="pytest -k expr" bash tools/gpu_ab.sh TAG [bench args...]
set -e
TAG=${1:-ab}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
if [ -n "$SEL" ]; then
  timeout -k 10 400 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 120 --timeout-method thread -k "$SEL" > $OUT/pytest_sel.log 2>&1 && echo "selected tests ok: $(tail -1 $OUT/pytest_sel.log)" || { echo "selected tests FAILED"; tail -40 $OUT/pytest_sel.log; exit 1; }
fi
# KNOB empty: each VALUES item is a comma-separated list of VAR=value assignments
for v in ${VALUES:-1}; do
  if [ -n "$KNOB" ]; then asg="$KNOB=$v"; else asg="${v//,/ }"; fi
  tag=$(echo "$v" | tr ',=' '__')
  env $asg timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu "$@" > $OUT/bench_$tag.log 2>&1 || { echo "bench $v FAILED"; tail -20 $OUT/bench_$tag.log; exit 1; }
  echo "$asg $(grep -o '"value": [0-9.]*' $OUT/bench_$tag.log) $(grep -o '"avg_launch_us": [0-9.]*' $OUT/bench_$tag.log)"
done
if [ -n "$DBG" ]; then
  env $DBG MADIPM_TREE_DEBUG=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu --no-opt "$@" > $OUT/tree_debug_bench.log 2> $OUT/tree_debug.txt && echo "tree debug ok" && head -30 $OUT/tree_debug.txt
fi
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-opt "$@" > $OUT/prof.log 2>&1 && echo "rocprof ok"
  python tools/prof_summary.py $OUT/prof > $OUT/prof_summary.txt 2>&1 || true
  head -25 $OUT/prof_summary.txt
fi
