#!/bin/bash
# r5 evidence 2: rocprofv3 kernel stats + one iteration's timeline (ex10, supportcase10, neos), PMC HBM
# traffic (ex10, neos), tree debug (ex10)
set -o pipefail
TAG=${1:?tag}
bash tools/gpu_prof.sh $TAG "ex10 supportcase10" 20 || exit 1
bash tools/gpu_prof.sh $TAG "neos" 4 || exit 1
bash tools/gpu_pmc.sh $TAG ex10 3 > /dev/null || exit 1
bash tools/gpu_pmc.sh $TAG neos 2 > /dev/null || exit 1
python3 - $TAG <<'PY'
import json, sys
t = sys.argv[1]
for c in ("ex10", "neos"):
    d = json.load(open(f"gpurun_out/{t}/{c}_pmc_traffic.json"))["kernels"]
    for k, v in sorted(d.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["dispatches"])[:6]:
        print(c, k, v["dispatches"], round(v["hbm_bytes_per_launch"] / 1e6, 1), round(v["hbm_bytes_lo_per_launch"] / 1e6, 1))
PY
bash tools/gpu_tree_debug.sh $TAG > /dev/null || exit 1
grep -E "tree fact|tree fwd|crit" gpurun_out/$TAG/tree_debug.txt | head -10
