#!/bin/bash
# Round evidence on one box: dense-QP bench with construction timings, rocprofv3 kernel stats and the
# iteration timeline of ex10 / supportcase10, and the PMC HBM traffic of ex10 (FETCH_SIZE and
# WRITE_SIZE in separate passes).  bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:?tag}; OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
MADIPM_SYMBOLIC_TIMING=1 timeout -k 10 600 python bench.py --config dense_qp --steps 2 --warmup 1 --no-cpu > $OUT/dense_qp_bench.log 2>&1 \
  || { echo "dense_qp bench FAILED"; tail -20 $OUT/dense_qp_bench.log; exit 1; }
tail -1 $OUT/dense_qp_bench.log | cut -c1-400
grep -E "^(setup_host|LDLSolver|symbolic)" $OUT/dense_qp_bench.log | head -40
bash tools/gpu_prof.sh $TAG "ex10 supportcase10" 6 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-opt --legs none > $OUT/pmc_$c.log 2>&1 \
    || { echo "pmc $c FAILED"; tail -20 $OUT/pmc_$c.log; exit 1; }
done
python3 tools/pmc_traffic.py $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE $OUT/pmc_traffic.json && head -c 1500 $OUT/pmc_traffic.json
