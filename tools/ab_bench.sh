#!/bin/bash
# A/B bench on the GPU box: GPU tests, then bench.py with an env toggle off/on.
# usage: bash tools/ab_bench.sh TAG ENVVAR [bench args...]
set -e
TAG=$1; VAR=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && echo "gpu tests ok" || { echo "gpu tests FAILED"; tail -30 $OUT/pytest_gpu.log; exit 1; }
env $VAR=0 timeout -k 10 300 python bench.py --no-cpu "$@" > $OUT/bench_off.log 2>&1 || { echo "bench off FAILED"; tail -20 $OUT/bench_off.log; exit 1; }
env $VAR=1 timeout -k 10 300 python bench.py --no-cpu "$@" > $OUT/bench_on.log 2>&1 || { echo "bench on FAILED"; tail -20 $OUT/bench_on.log; exit 1; }
python - $OUT <<'PY'
import json, sys
for k in ("off", "on"):
    d = json.loads(open(f"{sys.argv[1]}/bench_{k}.log").read().strip().splitlines()[-1])
    print(k, round(d["value"], 1), "iters/s", d["config"].get("status"), d["config"].get("iters_to_opt"), d["config"].get("objective"))
    print("   ", d["kernel_ms_warmup"])
PY
