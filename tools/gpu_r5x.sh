#!/bin/bash
# r5_x: loads issued unconditionally where a masked load serialised round trips (medium fronts' child
# adds, the forward tree's gather-slot destinations, fwd_init, the backward own values) — GPU tests,
# ex10 / supportcase10 benches, tree debug
set -o pipefail
TAG=${1:?tag}
SEL="tests/test_ldl_gpu.py tests/test_mpc_gpu.py tests/test_shard_gpu.py" STEPS=30 bash tools/gpu_ab.sh $TAG "MADIPM_BIG_SOLVE_WG=512" "ex10 supportcase10" || exit 1
for c in ex10 supportcase10; do tail -1 gpurun_out/$TAG/bench_${c}_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernel_ms_warmup',{}); print('$c', round(d['value'],1), round(d['roofline']['avg_launch_us'],1), k.get('k_fwd_tree'), k.get('k_bwd_tree'))"; done
bash tools/gpu_tree_debug.sh $TAG > /dev/null || exit 1
grep -E "tree fact|tree fwd|level 1: " gpurun_out/$TAG/tree_debug.txt | head -8
