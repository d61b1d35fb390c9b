#!/bin/bash
# r5_l: fold helpers (k_fact_tree) — GPU tests, ex10 / supportcase10 A/B (MADIPM_FOLD_HELP=0), tree debug
set -o pipefail
TAG=${1:?tag}
SEL="tests/test_ldl_gpu.py tests/test_mpc_gpu.py" STEPS=20 \
  bash tools/gpu_ab.sh $TAG "MADIPM_FOLD_HELP=0" "ex10 supportcase10" || exit 1
bash tools/gpu_tree_debug.sh $TAG > /dev/null || exit 1
grep -E "tree fact|crit|level [0-9]:  |fold level [12]" gpurun_out/$TAG/tree_debug.txt | head -24
