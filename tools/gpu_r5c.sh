#!/bin/bash
# r5 measurements: ex10 A/B of the partial-block count (single-workgroup finaliser), rocprof of ex10 /
# supportcase10 / neos, PMC traffic of ex10 and neos.  bash tools/gpu_r5c.sh TAG
set -o pipefail
TAG=${1:?tag}; OUT=gpurun_out/$TAG; mkdir -p $OUT
SEL=none STEPS=20 bash tools/gpu_ab.sh $TAG "MADIPM_PART_BLOCKS=1024 MADIPM_PART_BLOCKS=512" "ex10" || exit 1
bash tools/gpu_prof.sh $TAG "ex10 supportcase10 neos" 6 || exit 1
bash tools/gpu_pmc.sh $TAG ex10 3 || exit 1
bash tools/gpu_pmc.sh $TAG neos 2 || exit 1
