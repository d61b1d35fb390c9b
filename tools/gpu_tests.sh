#!/bin/bash
# GPU test subset with a per-step time limit: bash tools/gpu_tests.sh TAG "pytest selection" [limit_s]
# Output (with -s: the heartbeat lines of long tests reach the log) under gpurun_out/TAG/.
TAG=${1:?tag}; SEL=${2:?selection}; LIM=${3:-900}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 $LIM python -u -m pytest $SEL --maxfail=${MAXFAIL:-1} -v -s --timeout 900 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1
rc=$?; grep -E 'PASSED|FAILED|ERROR|passed|failed' $OUT/pytest.log | tail -40; exit $rc
