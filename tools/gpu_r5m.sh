#!/bin/bash
# r5_m: fold helper threshold A/B (MADIPM_FOLD_HELP_MIN 2 / 3 default / 4, off) on ex10 and supportcase10
set -o pipefail
TAG=${1:?tag}
SEL=none STEPS=30 bash tools/gpu_ab.sh $TAG "MADIPM_FOLD_HELP_MIN=2 MADIPM_FOLD_HELP_MIN=4 MADIPM_FOLD_HELP=0" "ex10" || exit 1
for E in MADIPM_FOLD_HELP_MIN=2 MADIPM_FOLD_HELP_MIN=3 MADIPM_FOLD_HELP_MIN=4 MADIPM_FOLD_HELP=0; do
  tail -1 gpurun_out/$TAG/bench_ex10_${E}.log 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$E', round(d['roofline']['avg_launch_us'],1))" || true
done
tail -1 gpurun_out/$TAG/bench_ex10_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', round(d['roofline']['avg_launch_us'],1))"
bash tools/gpu_tree_debug.sh $TAG > /dev/null || exit 1
grep -E "tree fact|crit|level [0-9]:  " gpurun_out/$TAG/tree_debug.txt | head -12
