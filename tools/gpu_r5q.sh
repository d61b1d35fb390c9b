#!/bin/bash
# r5_q: root solve loads (pivots before the barrier, 16 gather loads in flight) — GPU tests, ex10 x2 + profile
set -o pipefail
TAG=${1:?tag}
SEL="tests/test_ldl_gpu.py tests/test_mpc_gpu.py" STEPS=30 bash tools/gpu_ab.sh $TAG "MADIPM_BIG_SOLVE_WG=512" "ex10" || exit 1
bash tools/gpu_prof.sh $TAG "ex10" 20 || exit 1
