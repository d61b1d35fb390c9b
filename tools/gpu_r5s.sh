#!/bin/bash
# r5_s: root solve loads only (factor16r as committed) — mpc GPU tests, ex10
set -o pipefail
TAG=${1:?tag}
SEL="tests/test_mpc_gpu.py tests/test_ldl_gpu.py" STEPS=30 bash tools/gpu_ab.sh $TAG "MADIPM_BIG_SOLVE_WG=512" "ex10" || exit 1
