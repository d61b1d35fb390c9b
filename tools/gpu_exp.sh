#!/bin/bash
# Ad-hoc GPU experiments (run on the gpurun box from the repo root): microbenchmarks + bench sweeps of
# an environment knob.  usage: bash tools/gpu_exp.sh TAG
set -e
TAG=${1:-exp}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
if [ -x tools/final_bench ]; then timeout -k 10 60 tools/final_bench > $OUT/final_bench.txt 2>&1 && cat $OUT/final_bench.txt; fi
if [ -x tools/fetch_calib ]; then
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calib_fetch -o run -- tools/fetch_calib > $OUT/calib.log 2>&1 && echo "calib ok"
  timeout -s KILL 60 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/calib_trace -o run -- tools/fetch_calib >> $OUT/calib.log 2>&1 && echo "calib trace ok"
fi
for pb in ${PB_LIST:-2048 1024 512 256}; do
  MADIPM_PART_BLOCKS=$pb timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu > $OUT/bench_pb$pb.log 2>&1
  echo "part_blocks=$pb $(grep -o '"value": [0-9.]*' $OUT/bench_pb$pb.log)"
done
