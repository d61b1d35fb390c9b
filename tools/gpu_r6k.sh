#!/bin/bash
# k_fact_tree ticket order A/B (MADIPM_TREE_ORDER=1: list schedule): ldl GPU tests with it, ex10 and
# supportcase10 bench lines both ways, tree debug both ways
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG; mkdir -p $OUT
MADIPM_TREE_ORDER=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ldl_gpu.py -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for c in ex10 supportcase10; do
for E in 0 1 0 1; do
  MADIPM_TREE_ORDER=$E timeout -k 10 300 python bench.py --config $c --steps 30 --no-cpu --no-neos --no-highs --no-opt > $OUT/bench_${c}_$E.log 2>&1 || { tail -20 $OUT/bench_${c}_$E.log; exit 1; }
  tail -1 $OUT/bench_${c}_$E.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c order=$E', round(d['value'],1), round(d['roofline']['avg_launch_us'],1))"
done
done
for E in 0 1; do
  MADIPM_TREE_ORDER=$E bash tools/gpu_tree_debug.sh ${TAG}_o$E > /dev/null || exit 1
  grep -E "tree fact|crit" gpurun_out/${TAG}_o$E/tree_debug.txt | head -6
done
