#!/bin/bash
# r5_h .. r5_k: fold leaf-table prefetch + pivots in the L phase, leaf gather before the wait in k_fwd_tree,
# packed-lower tree U blocks, split-K k_big_upd128 on launches of few tiles — GPU tests, tree debug,
# benches (knob A/B), PMC, analysis timing
set -o pipefail
TAG=${1:?tag}
SEL="tests/test_ldl_gpu.py tests/test_shard_gpu.py tests/test_mpc_gpu.py tests/test_variants_gpu.py" STEPS=20 \
  bash tools/gpu_ab.sh $TAG "MADIPM_BIG_SOLVE_WG=512" "ex10" || exit 1
bash tools/gpu_tree_debug.sh $TAG > /dev/null || exit 1
grep -E "span|crit|fold level|level [0-9]:" gpurun_out/$TAG/tree_debug.txt | head -60
SEL=none STEPS=12 bash tools/gpu_ab.sh $TAG "MADIPM_UPD_SPLIT=0" "neos" || exit 1
SEL=none STEPS=12 bash tools/gpu_ab.sh $TAG "MADIPM_BIG_SOLVE_WG=512" "supportcase10" || exit 1
MADIPM_SYMBOLIC_TIMING=1 timeout -k 10 300 python bench.py --config ex10 --steps 2 --warmup 1 --no-cpu --no-opt --no-neos > gpurun_out/$TAG/ex10_symbolic_timing.log 2>&1 || exit 1
grep -E "symbolic|nd top|tables|analysis_s" gpurun_out/$TAG/ex10_symbolic_timing.log | head -40
bash tools/gpu_pmc.sh $TAG ex10 3 || exit 1
