#!/bin/bash
# Bench lines + rocprofv3 kernel stats for the non-headline BASELINE configs (supportcase10, neos stand-ins).
# usage: bash tools/gpu_configs.sh TAG
set -e
TAG=${1:-cfg}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python bench.py --config supportcase10 --steps 20 --warmup 2 --no-cpu > $OUT/supportcase10_bench.log 2>&1 && echo "sc10 ok" || { echo "sc10 FAILED"; tail -20 $OUT/supportcase10_bench.log; exit 1; }
tail -1 $OUT/supportcase10_bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_sc10 -o run -- python3 bench.py --config supportcase10 --steps 10 --warmup 1 --no-cpu --no-opt > $OUT/prof_sc10.log 2>&1 && echo "sc10 rocprof ok" || { echo "sc10 rocprof FAILED"; tail -20 $OUT/prof_sc10.log; exit 1; }
python tools/prof_summary.py $OUT/prof_sc10 > $OUT/supportcase10_prof_summary.txt 2>&1 || true
timeout -k 10 400 python bench.py --config neos --steps 8 --warmup 1 --no-cpu --no-opt > $OUT/neos_bench.log 2>&1 && echo "neos ok" || { echo "neos FAILED"; tail -20 $OUT/neos_bench.log; exit 1; }
tail -1 $OUT/neos_bench.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_neos -o run -- python3 bench.py --config neos --steps 4 --warmup 1 --no-cpu --no-opt > $OUT/prof_neos.log 2>&1 && echo "neos rocprof ok" || { echo "neos rocprof FAILED"; tail -20 $OUT/prof_neos.log; exit 1; }
python tools/prof_summary.py $OUT/prof_neos > $OUT/neos_prof_summary.txt 2>&1 || true
head -12 $OUT/neos_prof_summary.txt
