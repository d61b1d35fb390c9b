#!/bin/bash
# PMC HBM traffic per kernel (FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes) of a short bench:
#   bash tools/gpu_pmc.sh TAG CONFIG [steps]   -> gpurun_out/TAG/CONFIG_pmc_traffic.json
set -o pipefail
TAG=${1:?tag}; C=${2:-ex10}; S=${3:-3}; OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_${C}_$c -o run -- python3 bench.py --config $C --steps $S --warmup 1 --no-cpu --no-opt --legs none > $OUT/pmc_${C}_$c.log 2>&1 \
    || { echo "pmc $C $c FAILED"; tail -20 $OUT/pmc_${C}_$c.log; exit 1; }
done
python3 tools/pmc_traffic.py $OUT/pmc_${C}_FETCH_SIZE $OUT/pmc_${C}_WRITE_SIZE $OUT/${C}_pmc_traffic.json && head -c 1200 $OUT/${C}_pmc_traffic.json; echo
