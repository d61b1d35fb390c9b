#!/bin/bash
# A/B bench of library variants / env toggles on the GPU box (bench only, no tests):
#   bash tools/ab_variants.sh TAG "label|ENV=.. ENV2=.." ...   (MADIPM_LIB=... selects a variant build)
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for spec in "$@"; do
  label=${spec%%|*}; envs=${spec#*|}
  env $envs timeout -k 10 200 python bench.py --no-cpu --no-opt --legs none --steps 20 > $OUT/b_$label.log 2>&1 || { echo "$label FAILED"; tail -5 $OUT/b_$label.log; exit 1; }
  python - $OUT/b_$label.log $label <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:>10s} {d['value']:8.1f} iters/s  fact_tree {d['roofline']['avg_launch_us']:.1f} us  {d['kernel_ms_warmup']}")
PY
done
