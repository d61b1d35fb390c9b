#!/bin/bash
# r5_r: root solve loads (pivots before the barrier, 16 gather loads in flight); factor16r forms the
# next pivot, its reciprocal and column right after its first update — GPU tests, ex10 + neos, profile
set -o pipefail
TAG=${1:?tag}
SEL="tests/test_ldl_gpu.py tests/test_mpc_gpu.py tests/test_variants_gpu.py" STEPS=30 bash tools/gpu_ab.sh $TAG "MADIPM_BIG_SOLVE_WG=512" "ex10" || exit 1
SEL=none STEPS=12 bash tools/gpu_ab.sh $TAG "MADIPM_BIG_SOLVE_WG=512" "neos" || exit 1
bash tools/gpu_prof.sh $TAG "ex10" 20 || exit 1
bash tools/gpu_tree_debug.sh $TAG > /dev/null || exit 1
grep -E "tree fact|factor level [2-4]" gpurun_out/$TAG/tree_debug.txt | head -8
