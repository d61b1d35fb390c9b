#!/bin/bash
# windowed LDS source path (unsigned count) with one window in small launches: ldl GPU tests, bench lines
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ldl_gpu.py -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for c in ex10 supportcase10 neos ex10; do
  S=30; [ $c = neos ] && S=8
  timeout -k 10 300 python bench.py --config $c --steps $S --no-cpu --no-neos --no-highs --no-opt > $OUT/bench_$c.log 2>&1 || { tail -20 $OUT/bench_$c.log; exit 1; }
  tail -1 $OUT/bench_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', round(d['value'],2))"
done
bash tools/gpu_prof.sh $TAG "neos" 4 > /dev/null || exit 1
grep -E "k_assemble|k_asm|iteration" $OUT/neos_iter_timeline.txt | head -12
