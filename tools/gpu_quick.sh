#!/bin/bash
# Quick GPU iteration: parity tests, one bench line, stamps.  usage: tools/gpu_quick.sh TAG [pytest selector]
set -o pipefail
TAG=${1:-q}; SEL=${2:-tests}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest $SEL -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
&& timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 \
&& timeout -k 10 120 python tools/stamps.py 2000 > $OUT/stamps.log 2>&1
rc=$?
echo "exit $rc"
tail -5 $OUT/pytest_gpu.log
tail -1 $OUT/bench.log | cut -c1-600
cat $OUT/stamps.log
exit $rc
