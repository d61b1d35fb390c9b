#!/bin/bash
# r5_d: GPU tests of the solve / SpMV changes, then A/B of the SpMV next-row prefetch (ex10) and the
# big-front solve grid / panel-group knobs (neos).  bash tools/gpu_r5d.sh TAG
set -o pipefail
TAG=${1:?tag}
SEL="tests/test_ldl_gpu.py tests/test_mpc_gpu.py tests/test_mpc_paths_gpu.py tests/test_shard_gpu.py tests/test_kkt_ops_gpu.py" \
  STEPS=20 bash tools/gpu_ab.sh $TAG "MADIPM_SPMV_PF=0" "ex10" || exit 1
SEL=none STEPS=12 bash tools/gpu_ab.sh $TAG "MADIPM_BIG_SOLVE_WG=768 MADIPM_BIG_SOLVE_WG=1024 MADIPM_BIG_KPAN=6 MADIPM_BIG_KPAN=2" "neos" || exit 1
