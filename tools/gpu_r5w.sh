#!/bin/bash
# r5_w: medium fronts' child blocks added column-wise (lower triangle only) — GPU tests, supportcase10 +
# ex10 benches, supportcase10 tree debug
set -o pipefail
TAG=${1:?tag}
SEL="tests/test_ldl_gpu.py tests/test_mpc_gpu.py" STEPS=30 bash tools/gpu_ab.sh $TAG "MADIPM_BIG_SOLVE_WG=512" "supportcase10 ex10" || exit 1
for c in supportcase10 ex10; do tail -1 gpurun_out/$TAG/bench_${c}_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', round(d['value'],1), d['roofline']['kernel'], round(d['roofline']['avg_launch_us'],1))"; done
bash tools/gpu_tree_debug.sh $TAG --config supportcase10 > /dev/null || exit 1
grep -E "tree fact|crit|level [0-9]:  " gpurun_out/$TAG/tree_debug.txt | head -12
