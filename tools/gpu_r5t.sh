#!/bin/bash
# r5_t / r5_v: supportcase10 tree debug (the medium fronts' share of k_fact_tree)
set -o pipefail
TAG=${1:?tag}
bash tools/gpu_tree_debug.sh $TAG --config supportcase10 > /dev/null || exit 1
grep -vE "^/opt" gpurun_out/$TAG/tree_debug.txt | head -60
