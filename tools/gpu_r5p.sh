#!/bin/bash
# r5_p: big-child records a batch ahead in the assembly (one round trip per batch) — GPU tests
# (ldl, full-size neos), neos bench x2 + profile
set -o pipefail
TAG=${1:?tag}
SEL="tests/test_ldl_gpu.py tests/test_fullsize_gpu.py" STEPS=12 bash tools/gpu_ab.sh $TAG "MADIPM_BIG_SOLVE_WG=512" "neos" || exit 1
bash tools/gpu_prof.sh $TAG "neos" 4 || exit 1
