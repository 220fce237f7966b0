#!/bin/bash
# Round-end rehearsal of the driver's GPU steps: parity suite, smoke(), default bench.py.
set -o pipefail
TAG=${1:-chk}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
&& timeout -k 10 400 python bench.py > $OUT/bench_default.log 2>&1
rc=$?
tail -2 $OUT/pytest_gpu.log; cat $OUT/smoke.log; tail -1 $OUT/bench_default.log | cut -c1-400
exit $rc
