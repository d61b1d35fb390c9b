#!/bin/bash
# r5 evidence 3 (HEAD): the whole GPU suite, smoke(), the default bench line
set -o pipefail
TAG=${1:?tag}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1 \
  || { echo "pytest FAILED"; grep -E "FAILED|Error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke FAILED"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { echo "bench FAILED"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-600
