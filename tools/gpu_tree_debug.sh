#!/bin/bash
# Per-level phase timing of the tree kernels (MADIPM_TREE_DEBUG=1, wall clock inside the kernels) on
# the bench workload; run on the gpurun box from the repo root.  usage: bash tools/gpu_tree_debug.sh TAG [bench args]
set -e
TAG=${1:-dbg}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
MADIPM_TREE_DEBUG=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --no-opt --legs none "$@" > $OUT/tree_debug_bench.log 2> $OUT/tree_debug.txt && echo "tree debug ok" || { echo "tree debug FAILED"; tail -20 $OUT/tree_debug.txt; exit 1; }
head -60 $OUT/tree_debug.txt
