#!/bin/bash
# r5_n: fold helper share A/B (MADIPM_FOLD_HELP_SHARE quarters: 2 default, 3, 1) on ex10, twice
set -o pipefail
TAG=${1:?tag}
for rep in 1 2; do
  SEL=none STEPS=30 bash tools/gpu_ab.sh $TAG "MADIPM_FOLD_HELP_SHARE=3 MADIPM_FOLD_HELP_SHARE=1" "ex10" || exit 1
  for E in default MADIPM_FOLD_HELP_SHARE=3 MADIPM_FOLD_HELP_SHARE=1; do
    tail -1 gpurun_out/$TAG/bench_ex10_${E}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$E', round(d['value'],1), round(d['roofline']['avg_launch_us'],1))"
  done
done
