#!/bin/bash
# End-of-round evidence in one GPU session: full GPU parity suite, smoke(), the default bench
# line (C2 with CPU baseline, end-to-end and store-based compaction), then a rocprofv3 kernel
# trace of the same bench command.  Every GPU step has its own time limit; steps are chained.
# usage: tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
&& timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
&& timeout -k 10 420 python bench.py > $OUT/bench_c2.log 2>&1 \
&& timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $OUT/kt_c2 -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --no-e2e --no-compact --steps 5 --warmup 2 > $OUT/kt_c2.log 2>&1
rc=$?
tail -2 $OUT/pytest_gpu.log
tail -1 $OUT/smoke.log
tail -1 $OUT/bench_c2.log | cut -c1-300
echo "exit $rc"
exit $rc
