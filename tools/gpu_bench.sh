#!/bin/bash
# One bench line per config (no CPU baseline): bash tools/gpu_bench.sh TAG "cfg1 cfg2" [steps] [extra bench args]
TAG=${1:?tag}; CFGS=${2:-ex10}; S=${3:-20}; shift 3 || true
OUT=gpurun_out/$TAG; mkdir -p $OUT
for C in $CFGS; do
  timeout -k 10 400 python bench.py --config $C --steps $S --warmup 2 --no-cpu --legs none "$@" > $OUT/${C}_bench.log 2>&1 \
    || { echo "$C bench FAILED"; tail -30 $OUT/${C}_bench.log; exit 1; }
  tail -1 $OUT/${C}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$C', round(d['value'],2), 'iters/s', c.get('status'), c.get('iters_to_opt'), 'opt_s', c.get('wall_clock_to_opt_s'), 'dom', d['roofline']['kernel'], round(d['roofline']['avg_launch_us'],1), 'us', {k: v for k, v in list(d['kernel_ms_warmup'].items())[:8]})"
done
