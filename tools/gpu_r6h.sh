#!/bin/bash
# assembly entry count in the tile record: ldl GPU tests, ex10 rocprof, neos bench + rocprof
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ldl_gpu.py -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python bench.py --config neos --steps 8 --warmup 2 --no-cpu --no-neos --no-highs > $OUT/bench_neos.log 2>&1 || { tail -20 $OUT/bench_neos.log; exit 1; }
tail -1 $OUT/bench_neos.log | python3 -c "import json,sys,re; t=sys.stdin.read(); d=json.loads(t); print('neos', round(d['value'],2), re.findall(r'.analysis_s.: [0-9.]+', t)[:1])"
bash tools/gpu_prof.sh $TAG "ex10" 20 > /dev/null || exit 1
grep -E "k_assemble|k_asm_chunks|iteration" $OUT/ex10_prof_summary.txt $OUT/ex10_iter_timeline.txt | head -5
bash tools/gpu_prof.sh $TAG "neos" 4 > /dev/null || exit 1
grep -E "k_assemble|k_asm|iteration" $OUT/neos_iter_timeline.txt | head -12
