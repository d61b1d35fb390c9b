#!/bin/bash
# r5_k: split-K partial reload batched, factor16r next-pivot-first order — GPU tests, ex10 tree debug,
# neos A/B (split on / off) + neos kernel profile
set -o pipefail
TAG=${1:?tag}
SEL="tests/test_ldl_gpu.py tests/test_mpc_gpu.py tests/test_variants_gpu.py" STEPS=20 \
  bash tools/gpu_ab.sh $TAG "MADIPM_BIG_SOLVE_WG=512" "ex10" || exit 1
bash tools/gpu_tree_debug.sh $TAG > /dev/null || exit 1
grep -E "tree fact|crit|fold level [12]|factor level [1-4]" gpurun_out/$TAG/tree_debug.txt | head -14
SEL=none STEPS=12 bash tools/gpu_ab.sh $TAG "MADIPM_UPD_SPLIT=0" "neos" || exit 1
bash tools/gpu_prof.sh $TAG "neos" 4 || exit 1
