#!/bin/bash
# k_residual / k_eval row products with gdots: mpc + ldl GPU tests, ex10 bench x2, ex10 rocprof
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mpc_gpu.py tests/test_ldl_gpu.py -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for k in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --no-cpu --no-neos --no-highs --no-opt > $OUT/bench_ex10_$k.log 2>&1 || { tail -20 $OUT/bench_ex10_$k.log; exit 1; }
  tail -1 $OUT/bench_ex10_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ex10', round(d['value'],1), round(d['roofline']['avg_launch_us'],1))"
done
bash tools/gpu_prof.sh $TAG "ex10" 20 || exit 1
