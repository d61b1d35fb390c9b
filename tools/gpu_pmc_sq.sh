#!/bin/bash
# SQ counters of the bench's kernels, one --pmc pass per counter set (no trace domains):
#   bash tools/gpu_pmc_sq.sh TAG "C1 C2 ..." ["C1 ..."] ...   (env passes through, e.g. MADIPM_FOLD=0)
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-opt > $OUT/pmc$i.log 2>&1 && echo "pmc pass $i ok" || { echo "pmc pass $i FAILED"; tail -20 $OUT/pmc$i.log; exit 1; }
  python tools/pmc_sq.py $OUT/pmc$i/run_counter_collection.csv k_fact_tree k_small_blocked k_fwd_tree k_bwd_tree
done
