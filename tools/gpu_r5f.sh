#!/bin/bash
# r5_f: fused trsm tiles — GPU tests, then neos / dense QP A/B against MADIPM_FUSE_TRSM=0
set -o pipefail
TAG=${1:?tag}
SEL="tests/test_ldl_gpu.py tests/test_variants_gpu.py tests/test_shard_gpu.py tests/test_mpc_gpu.py" STEPS=12 \
  bash tools/gpu_ab.sh $TAG "MADIPM_FUSE_TRSM=0" "neos" || exit 1
SEL=none STEPS=3 bash tools/gpu_ab.sh $TAG "MADIPM_FUSE_TRSM=0" "dense_qp" || exit 1
