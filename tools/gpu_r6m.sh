#!/bin/bash
# assembly sources summed from LDS (MADIPM_ASM_LDS_SRC, default on): ldl GPU tests, neos / supportcase10 /
# ex10 bench lines both ways, neos rocprof timeline
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ldl_gpu.py -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for c in neos supportcase10 ex10; do
for E in 1 0 1 0; do
  S=30; [ $c = neos ] && S=8
  MADIPM_ASM_LDS_SRC=$E timeout -k 10 300 python bench.py --config $c --steps $S --no-cpu --no-neos --no-highs --no-opt > $OUT/bench_${c}_$E.log 2>&1 || { tail -20 $OUT/bench_${c}_$E.log; exit 1; }
  tail -1 $OUT/bench_${c}_$E.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c lds_src=$E', round(d['value'],2))"
done
done
bash tools/gpu_prof.sh $TAG "neos" 4 > /dev/null || exit 1
grep -E "k_assemble|k_asm|iteration" $OUT/neos_iter_timeline.txt | head -14
