#!/bin/bash
# r5_u: medium fronts — C of two tiles ahead in the trailing update, children's blocks added with every
# F load of a round in flight — GPU tests, supportcase10 bench x2 + tree debug, ex10
set -o pipefail
TAG=${1:?tag}
SEL="tests/test_ldl_gpu.py tests/test_mpc_gpu.py" STEPS=30 bash tools/gpu_ab.sh $TAG "MADIPM_BIG_SOLVE_WG=512" "supportcase10 ex10" || exit 1
for c in supportcase10 ex10; do tail -1 gpurun_out/$TAG/bench_${c}_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', round(d['value'],1), d['roofline']['kernel'], round(d['roofline']['avg_launch_us'],1))"; done
bash tools/gpu_tree_debug.sh $TAG --config supportcase10 > /dev/null || exit 1
grep -E "tree fact|crit" gpurun_out/$TAG/tree_debug.txt | head -4
