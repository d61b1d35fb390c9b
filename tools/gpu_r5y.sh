#!/bin/bash
# r5_y: fold-helper lookups hoisted to the front's start — GPU tests, ex10 x2, tree debug
set -o pipefail
TAG=${1:?tag}
SEL="tests/test_ldl_gpu.py tests/test_mpc_gpu.py" STEPS=30 bash tools/gpu_ab.sh $TAG "MADIPM_BIG_SOLVE_WG=512" "ex10" || exit 1
for E in default MADIPM_BIG_SOLVE_WG=512; do tail -1 gpurun_out/$TAG/bench_ex10_${E}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$E', round(d['value'],1), round(d['roofline']['avg_launch_us'],1))"; done
bash tools/gpu_tree_debug.sh $TAG > /dev/null || exit 1
grep -E "tree fact|crit" gpurun_out/$TAG/tree_debug.txt | head -6
