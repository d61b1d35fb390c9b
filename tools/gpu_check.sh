#!/bin/bash
# One GPU validation pass (run on the gpurun box from the repo root):
#   GPU parity tests -> full bench line (with cpu_baseline) -> rocprofv3 kernel stats of the bench.
# usage: bash tools/gpu_check.sh TAG [bench args...]
set -e
TAG=${1:-check}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && echo "gpu tests ok" || { echo "gpu tests FAILED"; tail -30 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 300 python bench.py "$@" > $OUT/bench.log 2>&1 && echo "bench ok" || { echo "bench FAILED"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-opt --legs none "$@" > $OUT/prof.log 2>&1 && echo "rocprof ok" || { echo "rocprof FAILED"; tail -30 $OUT/prof.log; exit 1; }
python tools/prof_summary.py $OUT/prof > $OUT/prof_summary.txt 2>&1 || true
head -25 $OUT/prof_summary.txt
# HBM traffic per kernel: FETCH_SIZE and WRITE_SIZE in separate --pmc passes (no trace domains)
if [ -n "$PMC" ]; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-opt --legs none "$@" > $OUT/pmc_fetch.log 2>&1 && echo "pmc fetch ok" || { echo "pmc fetch FAILED"; tail -20 $OUT/pmc_fetch.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-opt --legs none "$@" > $OUT/pmc_write.log 2>&1 && echo "pmc write ok" || { echo "pmc write FAILED"; tail -20 $OUT/pmc_write.log; exit 1; }
  python tools/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_traffic.json && echo "pmc traffic ok"
fi
