#!/bin/bash
# N back-to-back bench lines (no CPU leg) for run-to-run spread: bash tools/bench_repeat.sh TAG N [bench args...]
set -e
TAG=${1:-rep}; N=${2:-3}; shift 2 || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
for i in $(seq 1 $N); do
  timeout -k 10 300 python bench.py --no-cpu "$@" > $OUT/bench_rep$i.log 2>&1 || { echo "bench $i FAILED"; tail -20 $OUT/bench_rep$i.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('$OUT/bench_rep$i.log') if l.startswith('{')][-1]); print('rep $i', round(d['value'],1), 'iters/s', round(d['ms_per_step']*1000,1), 'us/iter')"
done
