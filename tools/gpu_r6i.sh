#!/bin/bash
# neos construction: symbolic stage times (MADIPM_SYMBOLIC_TIMING) and the bench's analysis_s
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG; mkdir -p $OUT
MADIPM_SYMBOLIC_TIMING=1 timeout -k 10 300 python bench.py --config neos --steps 2 --warmup 1 --no-cpu --no-neos --no-highs > $OUT/bench_neos.log 2> $OUT/neos_timing.log || { tail -20 $OUT/neos_timing.log; exit 1; }
grep -E "symbolic 1|10b|10a|symbolic 11|before 8 |nd top" $OUT/neos_timing.log | head -20
tail -1 $OUT/bench_neos.log | python3 -c "import json,sys,re; t=sys.stdin.read(); print(re.findall(r'.analysis_s.: [0-9.]+', t)[:1])"
python3 - <<'PY' > $OUT/ctor_split.txt 2>&1
import time, sys
sys.path.insert(0, "madipm.jl_amd")
import bench
from madipm_amd import MPCSolver
qp, _ = bench.build_problem("neos")
t = time.perf_counter(); s = MPCSolver(qp, **bench.solver_opts()); print("MPCSolver", round(time.perf_counter() - t, 3))
PY
cat $OUT/ctor_split.txt
