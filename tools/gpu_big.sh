#!/bin/bash
# Big-front configurations (neos, dense QP): bench line, rocprofv3 kernel stats and the MFMA
# PMC counters of the dense kernels (k_big_update, k_lb_syrk, k_big_trsm, ...), one pass per counter set.
# usage: bash tools/gpu_big.sh TAG [configs...]
set -e
TAG=${1:-big}; shift || true
CFGS=${@:-neos dense_qp}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for C in $CFGS; do
  S=8; [ "$C" = dense_qp ] && S=2
  timeout -k 10 500 python bench.py --config $C --steps $S --warmup 1 --no-cpu > $OUT/${C}_bench.log 2>&1 && echo "$C bench ok" || { echo "$C bench FAILED"; tail -20 $OUT/${C}_bench.log; exit 1; }
  tail -1 $OUT/${C}_bench.log | cut -c1-600
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$C -o run -- python3 bench.py --config $C --steps 2 --warmup 1 --no-cpu --no-opt > $OUT/prof_$C.log 2>&1 && echo "$C rocprof ok" || { echo "$C rocprof FAILED"; tail -20 $OUT/prof_$C.log; exit 1; }
  python tools/prof_summary.py $OUT/prof_$C > $OUT/${C}_prof_summary.txt 2>&1 || true
  head -14 $OUT/${C}_prof_summary.txt
  timeout -s KILL 500 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_mfma_$C -o run -- python3 bench.py --config $C --steps 1 --warmup 1 --no-cpu --no-opt > $OUT/pmc_mfma_$C.log 2>&1 && echo "$C pmc mfma ok" || { echo "$C pmc mfma FAILED"; tail -20 $OUT/pmc_mfma_$C.log; exit 1; }
done
