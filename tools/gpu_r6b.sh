#!/bin/bash
# neos assembly kernels: SQ / TA / TCP / TCC counters (one --pmc pass per set, no trace domains)
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES" \
           "TA_TA_BUSY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py --config neos --steps 2 --warmup 1 --no-cpu --no-opt --no-neos --no-highs > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i FAILED"; tail -20 $OUT/pmc$i.log; exit 1; }
  python3 tools/pmc_sq.py $OUT/pmc$i/run_counter_collection.csv k_assemble k_asm_update k_asm_chunks k_big_upd128 | tee $OUT/pmc$i.txt
done
