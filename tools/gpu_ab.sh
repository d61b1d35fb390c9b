#!/bin/bash
# A/B of environment knobs: GPU tests (default selection: ldl, mpc, mpc paths; SEL="..." overrides,
# SEL=none skips), then bench.py lines of each config with the default and with each knob.
#   bash tools/gpu_ab.sh TAG "KNOB=VAL KNOB2=VAL" "ex10 neos"
set -o pipefail
TAG=${1:?tag}; KNOBS=${2:?knobs}; CFGS=${3:-ex10}; OUT=gpurun_out/$TAG; mkdir -p $OUT
SEL=${SEL:-tests/test_ldl_gpu.py tests/test_mpc_gpu.py tests/test_mpc_paths_gpu.py}
STEPS=${STEPS:-20}
if [ "$SEL" != "none" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    $SEL > $OUT/pytest.log 2>&1 \
    || { echo "pytest FAILED"; grep -E "FAILED|Error|error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
for c in $CFGS; do
  for E in - $KNOBS; do
    [ "$E" = "-" ] && E=""
    env $E timeout -k 10 300 python bench.py --config $c --steps $STEPS --warmup 3 --no-cpu --legs none > $OUT/bench_${c}_${E:-default}.log 2>&1 \
      || { echo "bench $c ${E:-default} FAILED"; tail -20 $OUT/bench_${c}_${E:-default}.log; exit 1; }
    echo "$c ${E:-default}: $(tail -1 $OUT/bench_${c}_${E:-default}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(round(d["value"],1), round(d["ms_per_step"],4), c.get("status"), c.get("iters_to_opt"), c.get("wall_clock_to_opt_s"), c.get("objective"), c.get("analysis_s"))' 2>&1 | cut -c1-300)"
  done
done
