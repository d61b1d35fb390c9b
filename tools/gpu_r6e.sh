#!/bin/bash
# assembly from compact entry lists: ldl + mpc GPU tests, neos and ex10 bench lines, neos rocprof timeline
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ldl_gpu.py tests/test_mpc_gpu.py -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python bench.py --config neos --steps 8 --warmup 2 --no-cpu --no-neos --no-highs > $OUT/bench_neos.log 2>&1 || { tail -20 $OUT/bench_neos.log; exit 1; }
tail -1 $OUT/bench_neos.log | python3 -c "import json,sys,re; t=sys.stdin.read(); d=json.loads(t); print('neos', round(d['value'],2), re.findall(r'.analysis_s.: [0-9.]+', t)[:1])"
timeout -k 10 300 python bench.py --steps 30 --no-cpu --no-neos --no-highs --no-opt > $OUT/bench_ex10.log 2>&1 || { tail -20 $OUT/bench_ex10.log; exit 1; }
tail -1 $OUT/bench_ex10.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ex10', round(d['value'],1), round(d['roofline']['avg_launch_us'],1))"
bash tools/gpu_prof.sh $TAG "neos" 4 || exit 1
grep -E "k_assemble|k_asm" $OUT/neos_iter_timeline.txt
