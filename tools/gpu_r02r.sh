#!/bin/bash
# full GPU parity suite, then a rocprof kernel trace of one workload.  usage: tools/gpu_r02r.sh TAG WORKLOAD
set -o pipefail
TAG=${1:-r}; WL=${2:-c5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_$WL -o kt --output-format csv -- python3 bench.py --workload $WL --no-cpu-baseline --no-e2e --steps 5 --warmup 2 > $OUT/kt_$WL.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log; tail -1 $OUT/kt_$WL.log | cut -c1-400
exit $rc
