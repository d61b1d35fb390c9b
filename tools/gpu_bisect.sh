#!/bin/bash
# Run one pytest selection under several environment settings (A/B bisection of a failure):
#   bash tools/gpu_bisect.sh TAG "pytest selection" LIMIT_S "ENV1" "ENV2" ...   ("-" = no extra env)
# Stops at the first timeout / abort / crash (exit 124, 134, 137, 139).
TAG=${1:?tag}; SEL=${2:?selection}; LIM=${3:-300}; shift 3
OUT=gpurun_out/$TAG; mkdir -p $OUT
k=0
for E in "$@"; do
  k=$((k + 1))
  [ "$E" = "-" ] && E=""
  echo "== variant $k: ${E:-default}" | tee -a $OUT/bisect.log
  env $E timeout -k 10 $LIM python -u -m pytest $SEL -x -q --timeout 280 --timeout-method thread -m gpu > $OUT/v$k.log 2>&1
  rc=$?
  tail -30 $OUT/v$k.log | grep -E "passed|failed|Error|assert" | tail -8 | tee -a $OUT/bisect.log
  echo "rc $rc" | tee -a $OUT/bisect.log
  case $rc in 124|134|137|139) exit $rc;; esac
done
exit 0
